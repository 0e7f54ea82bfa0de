# round-2 GPU call AM: cfg2 eager vs graph under NERF_HEADS_SIDE (is the cfg3-graph loss of the split about graphs?)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02am
mkdir -p $OUT
for r in 1 2; do
  for hs in 1 0; do
    echo -n "heads_side=$hs " >> $OUT/ab.txt
    NERF_HEADS_SIDE=$hs timeout -k 10 300 python scripts/graph_ab.py --steps 30 --rounds 3 >> $OUT/ab.txt 2>/dev/null || exit 1
  done
done
cat $OUT/ab.txt
