#!/bin/bash
# (historical: the variant it measured was not kept and is no longer in the tree; result in DESIGN.md §5)
# dev (round 4, GPU box): the non-stem weight copies made on the side stream (engine prep_overlap):
# the whole GPU suite, then engine A/Bs at B=64 and B=256.
O=gpurun_out/r04prep
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || exit 1
timeout -k 10 500 python -u tools/engine_ab.py --batch 64 --cfg "" --cfg "prep_overlap=0" --cfg "" --cfg "prep_overlap=0" > $O/ab64.txt 2>&1 || exit 1
timeout -k 10 500 python -u tools/engine_ab.py --batch 256 --steps 5 --cfg "" --cfg "prep_overlap=0" --cfg "" --cfg "prep_overlap=0" > $O/ab256.txt 2>&1 || exit 1
