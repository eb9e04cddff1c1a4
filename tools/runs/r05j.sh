set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05k; mkdir -p $O
timeout -k 10 120 python -u tools/convbench.py --batch 64 --filter conv2 --reps 10 > $O/base.txt 2>&1
timeout -k 10 120 python -u tools/convbench.py --batch 256 --filter conv2 --reps 10 > $O/base256.txt 2>&1
for v in mfmaonly empty noepi ldsonly; do
  ARGUS_HIP_LIB=argus_amd/.variant/lib_$v.so timeout -k 10 120 python -u tools/convbench.py --batch 64 --filter conv2 --reps 10 > $O/$v.txt 2>&1 || echo "$v failed"
  ARGUS_HIP_LIB=argus_amd/.variant/lib_$v.so timeout -k 10 120 python -u tools/convbench.py --batch 256 --filter conv2 --reps 10 > $O/${v}256.txt 2>&1 || echo "$v failed"
done
for f in $O/*.txt; do echo "== $f"; grep "layer[123].[12].conv2" $f | cut -c1-150; done
