#!/bin/bash
# (historical: the variant it measured was not kept and is no longer in the tree; result in DESIGN.md §5)
# dev (round 4, GPU box): bn1 + ReLU applied in the 3x3 halo kernels' LDS (policy key 42, engine
# lds_prologue): halo parity tests first, then the whole GPU suite, a kernel trace, engine A/Bs.
O=gpurun_out/r04x
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 --timeout-method thread -k "halo" > $O/halo_tests.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-val-oracle --no-isolated > $O/tr.json 2>$O/tr.err || exit 1
python3 tools/profsum.py $O/tr/run_kernel_stats.csv 400 > $O/tr.sum 2>&1 || true
timeout -k 10 500 python -u tools/engine_ab.py --batch 64 --cfg "" --cfg "lds_prologue=0" --cfg "" --cfg "lds_prologue=0" > $O/ab64.txt 2>&1 || exit 1
timeout -k 10 500 python -u tools/engine_ab.py --batch 256 --steps 5 --cfg "" --cfg "lds_prologue=0" --cfg "" > $O/ab256.txt 2>&1 || exit 1
timeout -k 10 600 python -u tools/engine_ab.py --hw 376 672 --batch 128 --steps 5 --cfg "" --cfg "lds_prologue=0" --cfg "" > $O/ab376.txt 2>&1 || exit 1
