set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/prof_timeline.sh r05q_on > /dev/null 2>&1
bash tools/prof_timeline.sh r05q_off --tune 44=0 > /dev/null 2>&1
head -4 gpurun_out/tl_r05q_on/timeline.txt; head -4 gpurun_out/tl_r05q_off/timeline.txt
find gpurun_out/tl_r05q_* -name "*.csv" -delete
