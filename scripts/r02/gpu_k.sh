# round-2 GPU call K: eager vs hipGraph replay of the cfg2 step
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02k
mkdir -p $OUT
timeout -k 10 300 python -u scripts/graph_ab.py --steps 30 --rounds 3 > $OUT/graph_ab.json 2> $OUT/graph_ab.err; rc=$?
cat $OUT/graph_ab.json; tail -5 $OUT/graph_ab.err; exit $rc
