set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/profile_round.sh r05n
python3 tools/pmc_traffic.py gpurun_out/prof_r05n/pmc_fetch gpurun_out/prof_r05n/pmc_write gpurun_out/prof_r05n/pmc_traffic.json 64 256 256 bf16
python3 tools/profsum.py $(find gpurun_out/prof_r05n/stats -name "*kernel_stats.csv" | head -1) 60 > gpurun_out/prof_r05n/kernel_summary.txt
find gpurun_out/prof_r05n -name "*.csv" -size +2M -delete
head -70 gpurun_out/prof_r05n/kernel_summary.txt
