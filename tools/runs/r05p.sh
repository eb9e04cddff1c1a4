set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05p; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_train.py tests/test_gpu_parity.py -k "stats_only or side_stream_overlap or bf16_b64 or benched_kernel_selection" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -c PASSED $O/tests.log; tail -2 $O/tests.log
timeout -k 10 200 python -u tools/slack.py --batch 64 --steps 3 --streams main > $O/slack.txt 2>&1
grep "p1x1_fwd_stats\|3, 0>\|total" $O/slack.txt
timeout -k 10 400 python -u tools/engine_ab.py --batch 64 --steps 30 --rounds 3 --cfg "" --cfg "tune:44=0" > $O/ab.txt 2>&1
cat $O/ab.txt
