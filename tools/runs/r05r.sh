set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05r; mkdir -p $O
timeout -k 10 150 python -u tools/convbench.py --batch 64 --reps 10 > $O/base.txt 2>&1
for v in nomfma noload nobar nostore; do
  ARGUS_HIP_LIB=argus_amd/.variant/lib_w_$v.so timeout -k 10 150 python -u tools/convbench.py --batch 64 --reps 10 > $O/$v.txt 2>&1 || echo "$v failed"
done
for f in $O/*.txt; do echo "== $f"; grep "layer[1234].[01].conv[13]\|downsample" $f | sed 's/  p1:.*//' | cut -c1-40,100-200; done
