set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05w; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread tests/ -m gpu > $O/gpu_tests.log 2>&1; rc=$?
grep -c PASSED $O/gpu_tests.log; grep "FAILED\|ERROR" $O/gpu_tests.log | head; tail -2 $O/gpu_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
