#!/bin/bash
# PMC passes over one convbench layer filter: bash tools/pmc_layer.sh TAG FILTER [convbench args]
set -e
TAG=$1; FILT=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"
P2="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAIT_INST_LDS"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o run -- \
    python3 tools/convbench.py --filter $FILT --reps 3 "$@" > $O/p$i.log 2>&1
done
echo pmc done
