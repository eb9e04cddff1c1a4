set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "x8 or fp8_mx" > gpurun_out/r05h_tests.log 2>&1 || { tail -40 gpurun_out/r05h_tests.log; exit 1; }
tail -5 gpurun_out/r05h_tests.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "fp8" > gpurun_out/r05h_parity.log 2>&1 || { tail -40 gpurun_out/r05h_parity.log; exit 1; }
tail -5 gpurun_out/r05h_parity.log
timeout -k 10 400 python -u tools/engine_ab.py --batch 512 --dtype fp8 --steps 10 --rounds 2 --cfg "x8=0" --cfg "" --cfg "tune:37=10" --cfg "x8=0,tune:37=3" > gpurun_out/r05h_ab.txt 2>&1
cat gpurun_out/r05h_ab.txt
