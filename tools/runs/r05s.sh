set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05s; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "wgrad or stem or all_shapes or unstored" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -c PASSED $O/tests.log; tail -2 $O/tests.log
timeout -k 10 150 python -u tools/convbench.py --batch 64 --reps 10 > $O/convbench.txt 2>&1
timeout -k 10 400 python -u tools/engine_ab.py --batch 64 --steps 30 --rounds 2 --cfg "" > $O/ab.txt 2>&1
cat $O/ab.txt
timeout -k 10 200 python -u tools/slack.py --batch 64 --steps 3 --streams all > $O/slack.txt 2>&1
grep "wgrad\|total" $O/slack.txt
