set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05o; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_train.py tests/test_gpu_parity.py -k "apply_out or side_stream_overlap or bf16_b64 or x8" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -c PASSED $O/tests.log; tail -2 $O/tests.log
timeout -k 10 400 python -u tools/engine_ab.py --batch 64 --steps 30 --rounds 3 --cfg "" --cfg "a2_in_stats=0" > $O/ab.txt 2>&1
cat $O/ab.txt
