set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05t; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_model.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u tools/engine_ab.py --batch 64 --steps 30 --rounds 2 --cfg "" > $O/ab.txt 2>&1
cat $O/ab.txt
timeout -k 10 200 python -u tools/slack.py --batch 64 --steps 3 --streams main > $O/slack.txt 2>&1
head -25 $O/slack.txt
