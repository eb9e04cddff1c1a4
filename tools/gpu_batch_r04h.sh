#!/bin/bash
# (historical: the variant it measured was not kept and is no longer in the tree; result in DESIGN.md §5)
# dev (round 4, GPU box): XCD-contiguous pixel ranges in the max-pool forward / backward: stem tests,
# kernel times and FETCH/WRITE traffic of both max-pool kernels (new vs previous library), paired benches.
O=gpurun_out/r04mp
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "maxpool or stem" > $O/tests.txt 2>&1 || exit 1
for v in new old; do
  if [ $v = new ]; then L=argus_amd/libargus_hip.so; else L=argus_amd/.variant/libargus_hip_old.so; fi
  ARGUS_HIP_LIB=$L timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/st_$v -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-val-oracle --no-isolated > $O/st_$v.json 2>/dev/null || exit 1
  python3 tools/profsum.py $O/st_$v/run_kernel_stats.csv 400 > $O/st_$v.sum 2>&1 || true
  find $O/st_$v -name "*.csv" -size +2M -delete
  ARGUS_HIP_LIB=$L timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv -d $O/pmc_$v -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-val-oracle --no-isolated > $O/pmc_$v.json 2>/dev/null || exit 1
  python3 - $O/pmc_$v > $O/pmc_$v.txt <<'PY'
import csv, glob, sys, collections
tot = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "?")
        if "maxpool" in k:
            tot[k[:50]][r["Counter_Name"]] += float(r["Counter_Value"])
            n[(k[:50], r["Counter_Name"])] += 1
for k, d in tot.items():
    print(k, {c: round(v / n[(k, c)] / 1e6, 3) for c, v in d.items()}, "(M requests per launch)")
PY
  find $O/pmc_$v -name "*.csv" -size +2M -delete
done
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-val-oracle --no-isolated > $O/b64_new_$i.json 2>/dev/null || exit 1
  ARGUS_HIP_LIB=argus_amd/.variant/libargus_hip_old.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-val-oracle --no-isolated > $O/b64_old_$i.json 2>/dev/null || exit 1
done
