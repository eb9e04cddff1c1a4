#!/bin/bash
# dev: kernel tests for the changed kernels, then bench A/B over kernel-selection override sets
# (args: "k=v k=v" ...: argus_conv_policy_default keys; engine schedule switches: tools/engine_ab.py)
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
if [ -n "$KTESTS" ]; then
  timeout -k 10 300 $T tests/test_gpu_kernels.py -k "$KTESTS" > gpurun_out/ktests.log 2>&1 || { tail -30 gpurun_out/ktests.log; exit 1; }
  tail -1 gpurun_out/ktests.log
fi
i=0
for cfg in "$@"; do
  i=$((i+1)); tag="ab${i}_$(echo "$cfg" | tr ' =/' '___')"
  tunes="$cfg"
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-isolated --kernels $BENCH_ARGS ${tunes:+--tune $tunes} > gpurun_out/$tag.json 2> gpurun_out/$tag.err || { tail -20 gpurun_out/$tag.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('gpurun_out/$tag.json'));print('$tag', d['value'], d['ms_per_step'])"
done
