#!/bin/bash
# Round profile on the GPU box: kernel-trace stats, then separate FETCH_SIZE / WRITE_SIZE PMC passes.
#   bash tools/profile_round.sh TAG [bench args...]
# Outputs under gpurun_out/prof_TAG/ (copy the summaries into profiles/).
set -e
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- \
  python3 bench.py --no-cpu-baseline --no-val-oracle "$@" > $O/stats_bench.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- \
  python3 bench.py --no-cpu-baseline --no-val-oracle --steps 3 --warmup 1 "$@" > $O/fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- \
  python3 bench.py --no-cpu-baseline --no-val-oracle --steps 3 --warmup 1 "$@" > $O/write.log 2>&1
echo profile done
