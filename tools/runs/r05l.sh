set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05l; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "x8 or fp8_mx" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "fp8" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -3 $O/parity.log
timeout -k 10 200 python -u tools/slack.py --batch 512 --dtype fp8 --steps 2 --streams main --cfg "tune:37=10" > $O/slack_fp8_x8.txt 2>&1
grep "halo_kernel" $O/slack_fp8_x8.txt
timeout -k 10 500 python -u tools/engine_ab.py --batch 512 --dtype fp8 --steps 10 --rounds 3 --cfg "dtype=bf16" --cfg "" --cfg "tune:37=10" > $O/ab.txt 2>&1
cat $O/ab.txt
