#!/bin/bash
# dev (round 4, GPU box): halo weight-gradient split target (policy key 12) 128 vs the default 256,
# repeated at B=64 and B=256 (256x256 frames).
O=gpurun_out/r04k12
mkdir -p $O
timeout -k 10 500 python -u tools/engine_ab.py --batch 64 --cfg "" --cfg "tune:12=128" --cfg "" --cfg "tune:12=128" > $O/ab64.txt 2>&1 || exit 1
timeout -k 10 500 python -u tools/engine_ab.py --batch 256 --steps 5 --cfg "" --cfg "tune:12=128" --cfg "" --cfg "tune:12=128" > $O/ab256.txt 2>&1 || exit 1
