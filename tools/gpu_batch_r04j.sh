#!/bin/bash
# dev (round 4, GPU box): smallest K on the glds forward / dgrad kernel (policy key 8): 1024 (default)
# vs 512 / 256, engine A/B at B=64 and 376x672 B=128.
O=gpurun_out/r04k8
mkdir -p $O
timeout -k 10 500 python -u tools/engine_ab.py --batch 64 --cfg "" --cfg "tune:8=512" --cfg "tune:8=256" --cfg "" --cfg "tune:8=512" > $O/ab64.txt 2>&1 || exit 1
timeout -k 10 600 python -u tools/engine_ab.py --hw 376 672 --batch 128 --steps 5 --cfg "" --cfg "tune:8=512" --cfg "tune:8=256" > $O/ab376.txt 2>&1 || exit 1
