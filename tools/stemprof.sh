#!/bin/bash
# isolated stem wgrad timing (both kernels) + LDS / MFMA counters of the new one
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; export TMPDIR=/tmp
O=gpurun_out/stem_$1; mkdir -p $O
timeout -k 10 120 python3 -u tools/convbench.py --filter resnet.conv1 > $O/cb_on.txt 2>&1
timeout -k 10 120 python3 -u tools/convbench.py --filter resnet.conv1 --tune 34=0 > $O/cb_off.txt 2>&1
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d $O/p1 -o run -- python3 tools/convbench.py --filter resnet.conv1 --reps 2 > $O/p1.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pf -o run -- python3 tools/convbench.py --filter resnet.conv1 --reps 2 > $O/pf.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pw -o run -- python3 tools/convbench.py --filter resnet.conv1 --reps 2 > $O/pw.log 2>&1
cat $O/cb_on.txt $O/cb_off.txt
