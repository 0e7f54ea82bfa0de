# round-2 GPU call R: backward schedule A/B (weight-gradient side streams, tail on main)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02r
mkdir -p $OUT
timeout -k 10 400 python -u scripts/step_ab.py --steps 20 --rounds 3 --settings default side2 tail2 tail3 side2_tail2 > $OUT/step.json 2> $OUT/step.err; rc=$?
tail -1 $OUT/step.json; tail -3 $OUT/step.err; exit $rc
