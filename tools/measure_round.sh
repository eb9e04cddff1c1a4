#!/bin/bash
# Round measurement set on the GPU box (all outputs under gpurun_out/meas_TAG/), in two parts that
# each fit one gpurun call:   bash tools/measure_round.sh TAG a|b
#   a: bench lines for configs[1] (B=64) and the configs[2] per-rank point (B=256); B=64 kernel stats,
#      FETCH/WRITE PMC traffic, MFMA/wave-state counters and the step timeline
#   b: configs[3] (376x672, B=128) bench line + its kernel stats / PMC traffic / MFMA counters
#   c: configs[4]'s per-rank batch (B=512) in fp8 and bf16: PMC traffic + MFMA counters, bench lines
set -e
TAG=$1
PART=${2:-a}  # a | b | c
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/meas_$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
if [ "$PART" = a ]; then
  # counters first, so the bench lines below cite this round's PMC summaries (bench.py reads the newest
  # committed/copied profiles/*_pmc_*.json of the same workload)
  bash tools/profile_round.sh $TAG
  python3 tools/pmc_traffic.py gpurun_out/prof_$TAG/pmc_fetch gpurun_out/prof_$TAG/pmc_write $O/pmc_traffic.json 64 256 256 bf16
  python3 tools/profsum.py $(find gpurun_out/prof_$TAG/stats -name "*kernel_stats.csv" | head -1) 40 > $O/kernel_summary.txt
  cp $(find gpurun_out/prof_$TAG/stats -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv
  bash tools/prof_timeline.sh $TAG
  cp gpurun_out/tl_$TAG/timeline.txt $O/timeline.txt
  WORKLOAD="64 256 256 bf16" bash tools/prof_pmc.sh $TAG
  cp gpurun_out/pmc_$TAG/summary.json $O/pmc_mfma_summary.json
  cp gpurun_out/pmc_$TAG/summary.txt $O/pmc_mfma_summary.txt
  cp $O/pmc_traffic.json profiles/${TAG}_pmc_traffic.json
  cp $O/pmc_mfma_summary.json profiles/${TAG}_pmc_mfma_summary.json
  timeout -k 10 240 python3 -u bench.py > $O/bench.json 2> $O/bench.err
  timeout -k 10 180 python3 -u bench.py --batch 256 --no-cpu-baseline > $O/bench_b256.json 2> $O/bench_b256.err
elif [ "$PART" = c ]; then
  # configs[4]'s per-rank batch (B=512): PMC traffic and MFMA counters for fp8 and bf16, then the lines
  for DT in fp8 bf16; do
    bash tools/profile_round.sh ${TAG}_b512_$DT --batch 512 --dtype $DT --steps 3 --warmup 1 --no-isolated
    python3 tools/pmc_traffic.py gpurun_out/prof_${TAG}_b512_$DT/pmc_fetch gpurun_out/prof_${TAG}_b512_$DT/pmc_write \
      $O/pmc_traffic_b512_$DT.json 512 256 256 $DT
    WORKLOAD="512 256 256 $DT" bash tools/prof_pmc.sh ${TAG}_b512_$DT --batch 512 --dtype $DT
    cp gpurun_out/pmc_${TAG}_b512_$DT/summary.json profiles/${TAG}_b512_${DT}_pmc_mfma_summary.json
    cp gpurun_out/pmc_${TAG}_b512_$DT/summary.txt $O/b512_${DT}_pmc_mfma_summary.txt
    cp $O/pmc_traffic_b512_$DT.json profiles/${TAG}_b512_${DT}_pmc_traffic.json
    python3 tools/profsum.py $(find gpurun_out/prof_${TAG}_b512_$DT/stats -name "*kernel_stats.csv" | head -1) 30 \
      > $O/b512_${DT}_kernel_summary.txt
    # keep the merge-back small: the B=512 traces and counter dumps are summarised above
    find gpurun_out/prof_${TAG}_b512_$DT gpurun_out/pmc_${TAG}_b512_$DT -name "*.csv" -size +2M -delete
  done
  timeout -k 10 240 python3 -u bench.py --dtype fp8 --batch 512 --no-cpu-baseline --steps 5 --warmup 2 \
    > $O/bench_b512_fp8.json 2> $O/bench_b512_fp8.err
  timeout -k 10 240 python3 -u bench.py --batch 512 --no-cpu-baseline --steps 5 --warmup 2 \
    > $O/bench_b512_bf16.json 2> $O/bench_b512_bf16.err
else
  bash tools/profile_round.sh ${TAG}_376 --hw 376 672 --batch 128 --steps 5 --warmup 2
  python3 tools/pmc_traffic.py gpurun_out/prof_${TAG}_376/pmc_fetch gpurun_out/prof_${TAG}_376/pmc_write $O/pmc_traffic_376x672.json 128 376 672 bf16
  WORKLOAD="128 376 672 bf16" bash tools/prof_pmc.sh ${TAG}_376 --hw 376 672 --batch 128
  cp gpurun_out/pmc_${TAG}_376/summary.json $O/376x672_pmc_mfma_summary.json
  cp gpurun_out/pmc_${TAG}_376/summary.txt $O/376x672_pmc_mfma_summary.txt
  cp $O/pmc_traffic_376x672.json profiles/${TAG}_376x672_pmc_traffic.json
  cp $O/376x672_pmc_mfma_summary.json profiles/${TAG}_376x672_pmc_mfma_summary.json
  timeout -k 10 240 python3 -u bench.py --hw 376 672 --batch 128 --no-cpu-baseline --kernels \
    > $O/bench_376x672.json 2> $O/bench_376x672_kernels.txt
fi
echo "measure $PART done"
