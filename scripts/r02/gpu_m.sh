# round-2 GPU call M: side-stream priority A/B on the cfg2 step (TN pipeline depth 1 and 3)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02m
mkdir -p $OUT
for ns in 1 3; do
  NERF_TN_NS=$ns timeout -k 10 300 python -u scripts/step_ab.py --steps 20 --rounds 3 --settings default side_hi > $OUT/step_ns$ns.json 2> $OUT/step_ns$ns.err || exit 1
  echo "ns=$ns"; tail -1 $OUT/step_ns$ns.json
done
