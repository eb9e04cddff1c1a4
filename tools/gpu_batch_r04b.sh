#!/bin/bash
# dev (round 4, GPU box): maxpool-backward grid cap (ARGUS_MPB_BLOCKS) — stem parity tests on the new
# library, per-kernel times of maxpool_bwd + the stem bwd_finalize for 2048 / 8192 / 1024 blocks, then
# paired B=64 benches (new vs 8192) in the same instance.
O=gpurun_out/r04v
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "maxpool or stem" > $O/tests.txt 2>&1 || exit 1
for v in new mpb8192 mpb1024; do
  if [ $v = new ]; then L=argus_amd/libargus_hip.so; else L=argus_amd/.variant/libargus_hip_$v.so; fi
  ARGUS_HIP_LIB=$L timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-val-oracle --no-isolated > $O/$v.json 2>$O/$v.err || exit 1
  python3 tools/profsum.py $(ls $O/$v/*/run_kernel_stats.csv $O/$v/run_kernel_stats.csv 2>/dev/null | head -n1) 400 > $O/$v.sum 2>&1 || true
  find $O/$v -name "*.csv" -size +2M -delete
done
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-val-oracle --no-isolated > $O/pair_new_$i.json 2>/dev/null || exit 1
  ARGUS_HIP_LIB=argus_amd/.variant/libargus_hip_mpb8192.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-val-oracle --no-isolated > $O/pair_8192_$i.json 2>/dev/null || exit 1
done
