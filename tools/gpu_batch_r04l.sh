#!/bin/bash
# dev (round 4, GPU box): 8 group results in flight per lane in the BN finalize's second level
# (merge_groups): BN tests, finalize kernel times (new vs previous library), paired B=64 benches.
O=gpurun_out/r04fin
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "bn or finalize or stem" > $O/tests.txt 2>&1 || exit 1
for v in new old; do
  if [ $v = new ]; then L=argus_amd/libargus_hip.so; else L=argus_amd/.variant/libargus_hip_old.so; fi
  ARGUS_HIP_LIB=$L timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/st_$v -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-val-oracle --no-isolated > $O/st_$v.json 2>/dev/null || exit 1
  python3 tools/profsum.py $O/st_$v/run_kernel_stats.csv 400 > $O/st_$v.sum 2>&1 || true
  find $O/st_$v -name "*.csv" -size +2M -delete
done
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-val-oracle --no-isolated > $O/b64_new_$i.json 2>/dev/null || exit 1
  ARGUS_HIP_LIB=argus_amd/.variant/libargus_hip_old.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-val-oracle --no-isolated > $O/b64_old_$i.json 2>/dev/null || exit 1
done
