set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 bash tools/measure_round.sh r05z a > gpurun_out/r05z_a.log 2>&1 || { tail -20 gpurun_out/r05z_a.log; exit 1; }
find gpurun_out/prof_r05z gpurun_out/pmc_r05z gpurun_out/tl_r05z -name "*.csv" -size +2M -delete
tail -1 gpurun_out/meas_r05z/bench.json | cut -c1-400
tail -1 gpurun_out/meas_r05z/bench_b256.json | cut -c1-300
