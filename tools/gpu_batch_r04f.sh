#!/bin/bash
# (historical: the variant it measured was not kept and is no longer in the tree; result in DESIGN.md §5)
# dev (round 4, GPU box): 32-pixel k-steps for the bf16 128x128 weight gradient (ARGUS_WG128_BKP32:
# 32 KB LDS, three workgroups per CU): weight-gradient parity tests on the variant library, then paired
# benches (default vs variant) in one instance.
O=gpurun_out/r04z
mkdir -p $O
export TMPDIR=/tmp
V=argus_amd/.variant/libargus_hip_bkp32.so
ARGUS_HIP_LIB=$V timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wgrad or all_shapes or selection or b64" > $O/tests_variant.txt 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-val-oracle --no-isolated > $O/b64_def_$i.json 2>/dev/null || exit 1
  ARGUS_HIP_LIB=$V timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-val-oracle --no-isolated > $O/b64_var_$i.json 2>/dev/null || exit 1
done
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --batch 256 --steps 5 --warmup 2 --no-cpu-baseline --no-val-oracle --no-isolated > $O/b256_def_$i.json 2>/dev/null || exit 1
  ARGUS_HIP_LIB=$V timeout -k 10 200 python -u bench.py --batch 256 --steps 5 --warmup 2 --no-cpu-baseline --no-val-oracle --no-isolated > $O/b256_var_$i.json 2>/dev/null || exit 1
  timeout -k 10 200 python -u bench.py --hw 376 672 --batch 128 --steps 5 --warmup 2 --no-cpu-baseline --no-val-oracle --no-isolated > $O/b376_def_$i.json 2>/dev/null || exit 1
  ARGUS_HIP_LIB=$V timeout -k 10 200 python -u bench.py --hw 376 672 --batch 128 --steps 5 --warmup 2 --no-cpu-baseline --no-val-oracle --no-isolated > $O/b376_var_$i.json 2>/dev/null || exit 1
done
