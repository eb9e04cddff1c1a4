set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 bash tools/measure_round.sh r05z b > gpurun_out/r05z_b.log 2>&1 || { tail -20 gpurun_out/r05z_b.log; exit 1; }
find gpurun_out/prof_r05z_376 gpurun_out/pmc_r05z_376 -name "*.csv" -size +2M -delete
tail -1 gpurun_out/meas_r05z/bench_376x672.json | cut -c1-300
timeout -k 10 1000 bash tools/measure_round.sh r05z c > gpurun_out/r05z_c.log 2>&1 || { tail -20 gpurun_out/r05z_c.log; exit 1; }
tail -1 gpurun_out/meas_r05z/bench_b512_fp8.json | cut -c1-300
tail -1 gpurun_out/meas_r05z/bench_b512_bf16.json | cut -c1-300
