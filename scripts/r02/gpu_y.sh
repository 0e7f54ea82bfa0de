# round-2 GPU call Y: tail layers' weight gradients behind one wait (NERF_TAIL_SIDE) A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02y
mkdir -p $OUT
timeout -k 10 500 python -u scripts/step_ab.py --steps 20 --rounds 6 --settings default slab_stream tail1_ts2 > $OUT/step.json 2> $OUT/step.err; rc=$?
tail -1 $OUT/step.json; exit $rc
