#!/bin/bash
# dev (round 4, GPU box): maxpool backward reduction planes padded (LDS bank conflicts): stem tests,
# one PMC pass (LDS conflict counters) and a kernel trace of a short B=64 bench.
O=gpurun_out/r04y
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "maxpool or stem" > $O/tests.txt 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES --output-format csv -d $O/pmc -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-val-oracle --no-isolated > $O/pmc.json 2>$O/pmc.err || exit 1
python3 - $O <<'PY' > $O/maxpool_lds.txt
import csv, glob, sys, collections
O = sys.argv[1]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(O + "/pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "?")
        if "maxpool" in k or "bn_apply" in k:
            tot[k[:60]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in tot.items():
    c, a = d.get("SQ_LDS_BANK_CONFLICT", 0), d.get("SQ_LDS_IDX_ACTIVE", 0)
    print(f"{k:60s} conflict/active {c / a if a else float('nan'):.3f}  " + " ".join(f"{n}={v:.4g}" for n, v in sorted(d.items())))
PY
find $O/pmc -name "*.csv" -size +2M -delete
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-val-oracle --no-isolated > $O/tr.json 2>$O/tr.err || exit 1
python3 tools/profsum.py $O/tr/run_kernel_stats.csv 400 > $O/tr.sum 2>&1 || true
find $O/tr -name "*.csv" -size +2M -delete
