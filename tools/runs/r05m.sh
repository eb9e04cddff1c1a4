set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05m; mkdir -p $O
timeout -k 10 200 python -u tools/slack.py --batch 64 --steps 3 --streams main,all > $O/slack_b64.txt 2>&1
timeout -k 10 200 python -u tools/slack.py --batch 64 --steps 3 --streams main --cfg "wgrad_overlap=0" > $O/slack_b64_serial.txt 2>&1
timeout -k 10 200 python -u tools/engine_ab.py --batch 64 --steps 20 --rounds 2 --cfg "" --cfg "wgrad_overlap=0" > $O/ab.txt 2>&1
cat $O/ab.txt
