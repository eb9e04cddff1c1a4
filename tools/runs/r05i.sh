set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/slack.py --batch 512 --dtype fp8 --steps 2 --streams main --cfg "x8=0" > gpurun_out/r05i_slack_fp8_x8off.txt 2>&1
timeout -k 10 200 python -u tools/slack.py --batch 512 --dtype fp8 --steps 2 --streams main --cfg "tune:37=10" > gpurun_out/r05i_slack_fp8_x8.txt 2>&1
timeout -k 10 200 python -u tools/slack.py --batch 512 --dtype bf16 --steps 2 --streams main > gpurun_out/r05i_slack_bf16.txt 2>&1
grep -h "halo_kernel\|total\|==" gpurun_out/r05i_slack_*.txt
