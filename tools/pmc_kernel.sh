#!/bin/bash
# dev (GPU box): kernel-trace stats + three PMC passes over one convbench layer filter, then the
# per-kernel counter table.   bash tools/pmc_kernel.sh TAG FILTER [convbench args]
set -e
TAG=$1; FILT=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmck_$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/st -o run -- \
  python3 tools/convbench.py --filter $FILT --reps 3 "$@" > $O/st.log 2>&1
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM"
P3="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_WAVES_EQ_64 SQ_INSTS_BRANCH"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o run -- \
    python3 tools/convbench.py --filter $FILT --reps 3 "$@" > $O/p$i.log 2>&1
done
python3 - "$O" <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for f in glob.glob(O + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "?")[:70]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
for f in glob.glob(O + "/st/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print("stats", r["Name"][:70], r["Calls"], r["AverageNs"])
for k, d in tot.items():
    print("==", k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {v:.4g}")
PY
