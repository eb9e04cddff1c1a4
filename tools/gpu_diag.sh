#!/bin/bash
# dev: A/B benches, then the GPU suite in the background while rocm-smi samples the GPU at the hang point
mkdir -p gpurun_out
bash tools/gpu_ab.sh "$@" || exit 1
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/diag_tests.log 2>&1 &
P=$!
for i in $(seq 1 14); do
  sleep 20
  echo "t=$((i*20)) $(grep -c PASSED gpurun_out/diag_tests.log) $(tail -c 120 gpurun_out/diag_tests.log | tr '\n' ' ')" >> gpurun_out/diag_smi.txt
  rocm-smi --showuse --showmemuse 2>/dev/null | grep -E "GPU use|Memory Activity|GPU Memory Allocated" >> gpurun_out/diag_smi.txt
  kill -0 $P 2>/dev/null || break
done
wait $P; rc=$?
grep -E "passed|failed|Timeout" gpurun_out/diag_tests.log | tail -3
exit $rc
