#!/bin/bash
# dev: run GPU steps in order, each under its own time limit; stop at the first crash / timeout / abort
# (test failures are reported and the next step still runs). Usage:
#   bash tools/gpu_steps.sh "SECONDS:LOG:COMMAND" ...
mkdir -p gpurun_out
rc_all=0
for step in "$@"; do
  secs=${step%%:*}; rest=${step#*:}; log=${rest%%:*}; cmd=${rest#*:}
  echo "== [$secs s] $cmd  > gpurun_out/$log"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$log" 2>&1
  rc=$?
  tail -4 "gpurun_out/$log"
  echo "== rc=$rc"
  case $rc in
    0) ;;
    124|137|134|139|143) echo "== stopping: GPU step crashed or timed out"; exit $rc ;;
    *) rc_all=$rc ;;
  esac
done
exit $rc_all
