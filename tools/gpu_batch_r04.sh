#!/bin/bash
# dev (round 4, GPU box): engine A/B runs of the schedule / policy variants and paired bench runs against
# variant libraries built on the CPU side (argus_amd/.variant/: wgrad occupancy 3).
# (at most 3 model instances per 376x672 B=128 A/B: five ran the 288 GB card out of memory)
mkdir -p gpurun_out/r04u
timeout -k 10 400 python -u tools/engine_ab.py --batch 64 --cfg "" --cfg "tune:14=64" --cfg "" --cfg "tune:14=16" --cfg "tune:14=64" > gpurun_out/r04u/ab64.txt 2>&1 || exit 1
timeout -k 10 400 python -u tools/engine_ab.py --batch 256 --steps 5 --cfg "" --cfg "tune:14=64" --cfg "" > gpurun_out/r04u/ab256.txt 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --hw 376 672 --batch 128 --steps 5 --warmup 2 --no-cpu-baseline --no-val-oracle --no-isolated > gpurun_out/r04u/new376_$i.json 2>/dev/null || exit 1
  ARGUS_HIP_LIB=argus_amd/.variant/libargus_hip_occ3.so timeout -k 10 200 python -u bench.py --hw 376 672 --batch 128 --steps 5 --warmup 2 --no-cpu-baseline --no-val-oracle --no-isolated > gpurun_out/r04u/occ3_376_$i.json 2>/dev/null || exit 1
  timeout -k 10 200 python -u bench.py --batch 256 --steps 5 --warmup 2 --no-cpu-baseline --no-val-oracle --no-isolated > gpurun_out/r04u/new256_$i.json 2>/dev/null || exit 1
  ARGUS_HIP_LIB=argus_amd/.variant/libargus_hip_occ3.so timeout -k 10 200 python -u bench.py --batch 256 --steps 5 --warmup 2 --no-cpu-baseline --no-val-oracle --no-isolated > gpurun_out/r04u/occ3_256_$i.json 2>/dev/null || exit 1
done
