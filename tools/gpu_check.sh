#!/bin/bash
# dev: full GPU test suite + smoke + bench at HEAD, then optional bench A/B over tuning-key sets ("k=v ...")
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { grep -E "FAILED|Error|Timeout" gpurun_out/gpu_tests.log | head; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
bash tools/gpu_ab.sh "" "$@"
