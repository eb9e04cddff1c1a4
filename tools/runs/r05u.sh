set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05u; mkdir -p $O
timeout -k 10 600 python -u tools/engine_ab.py --batch 64 --steps 30 --rounds 3 --cfg "" --cfg "tune:38=1" --cfg "tune:42=3" --cfg "tune:43=0" > $O/ab.txt 2>&1
cat $O/ab.txt
