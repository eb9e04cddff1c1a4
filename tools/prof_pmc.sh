#!/bin/bash
# MFMA / wave-state / LDS counters of a short bench run, one rocprofv3 --pmc pass each (<= 8 SQ + 1 GRBM),
# then tools/pmc_summary.py.   bash tools/prof_pmc.sh TAG [bench args...]   (GPU box)
set -e
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o run -- \
    python3 bench.py --no-cpu-baseline --no-val-oracle --no-isolated --steps 2 --warmup 1 "$@" > $O/p$i.log 2>&1
done
python3 tools/pmc_summary.py $O/summary.json $O/p1 $O/p2 --workload ${WORKLOAD:-64 256 256 bf16} > $O/summary.txt
echo pmc done
