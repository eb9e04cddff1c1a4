#!/bin/bash
# (historical: the variant it measured was not kept and is no longer in the tree; result in DESIGN.md §5)
# dev (round 4, GPU box): elementwise-pass geometry (bn_apply / bn_bwd_apply ...): workgroup target
# 512 (default) / 1024 / 2048 and 8 pixels in flight per thread, paired benches in one instance.
O=gpurun_out/r04ew
mkdir -p $O
export TMPDIR=/tmp
run() {  # name lib args...
  local n=$1 l=$2; shift 2
  if [ "$l" = def ]; then timeout -k 10 200 python -u bench.py "$@" --no-cpu-baseline --no-val-oracle --no-isolated > $O/$n.json 2>/dev/null
  else ARGUS_HIP_LIB=argus_amd/.variant/libargus_hip_$l.so timeout -k 10 200 python -u bench.py "$@" --no-cpu-baseline --no-val-oracle --no-isolated > $O/$n.json 2>/dev/null; fi
}
for i in 1 2; do
  for l in def t1024 t2048 u8; do run b64_${l}_$i $l --steps 20 --warmup 5 || exit 1; done
done
for l in def t2048 u8 def; do run b256_${l}_$RANDOM $l --batch 256 --steps 5 --warmup 2 || exit 1; done
