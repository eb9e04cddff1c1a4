#!/bin/bash
# Kernel trace of a short bench run + timeline breakdown + the list of PMC counters on this GPU.
#   bash tools/prof_timeline.sh TAG [bench args...]      (run on the GPU box)
set -e
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/tl_$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 bench.py --no-cpu-baseline --no-val-oracle --no-isolated --steps 10 --warmup 3 "$@" > $O/bench.log 2>&1
python3 tools/timeline.py $(find $O/trace -name "*kernel_trace.csv" | head -1) --steps 8 --first 10 --list > $O/timeline.txt
echo timeline done
