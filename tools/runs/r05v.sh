set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05v; mkdir -p $O
timeout -k 10 500 python -u tools/engine_ab.py --batch 64 --steps 30 --rounds 3 --cfg "" --cfg "tune:38=1" > $O/ab64.txt 2>&1
cat $O/ab64.txt
timeout -k 10 500 python -u tools/engine_ab.py --batch 256 --steps 10 --rounds 2 --cfg "" --cfg "tune:38=1" > $O/ab256.txt 2>&1
cat $O/ab256.txt
timeout -k 10 500 python -u tools/engine_ab.py --batch 128 --hw 376 672 --steps 6 --rounds 2 --cfg "" --cfg "tune:38=1" > $O/ab376.txt 2>&1
cat $O/ab376.txt
