#!/bin/bash
# dev (round 4, GPU box): kernel tests of the changed kernels, the GPU suite, engine A/B runs of the
# schedule / policy variants and paired bench runs against the kLoadBatch=1 variant library
# (argus_amd/.variant/libargus_hip_lb1.so, built on the CPU side).
mkdir -p gpurun_out/r04s
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "se3 or loss or fused_dgrad or maxpool or stem_backward" > gpurun_out/r04s/k.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04s/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 400 python -u tools/engine_ab.py --batch 64 --cfg "" --cfg "fuse_dgw=0" --cfg "tune:39=0" --cfg "tune:40=0" --cfg "tune:39=0,tune:40=0" --cfg "tune:6=256,tune:27=256,tune:39=0" --cfg "tune:6=256,tune:27=256,tune:39=0,tune:40=0" --cfg "" > gpurun_out/r04s/ab64.txt 2>&1 || exit 1
timeout -k 10 400 python -u tools/engine_ab.py --batch 128 --hw 376 672 --steps 5 --cfg "" --cfg "tune:39=0" --cfg "tune:40=0" --cfg "tune:14=64" --cfg "tune:6=256,tune:27=256,tune:39=0" --cfg "" > gpurun_out/r04s/ab376.txt 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-val-oracle --no-isolated > gpurun_out/r04s/new$i.json 2>/dev/null || exit 1
  ARGUS_HIP_LIB=argus_amd/.variant/libargus_hip_lb1.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-val-oracle --no-isolated > gpurun_out/r04s/lb1_$i.json 2>/dev/null || exit 1
  ARGUS_HIP_LIB=argus_amd/.variant/libargus_hip_occ3.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-val-oracle --no-isolated > gpurun_out/r04s/occ3_$i.json 2>/dev/null || exit 1
done
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --hw 376 672 --batch 128 --steps 5 --warmup 2 --no-cpu-baseline --no-val-oracle --no-isolated > gpurun_out/r04s/new376_$i.json 2>/dev/null || exit 1
  ARGUS_HIP_LIB=argus_amd/.variant/libargus_hip_occ3.so timeout -k 10 200 python -u bench.py --hw 376 672 --batch 128 --steps 5 --warmup 2 --no-cpu-baseline --no-val-oracle --no-isolated > gpurun_out/r04s/occ3_376_$i.json 2>/dev/null || exit 1
done
