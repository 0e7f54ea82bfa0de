# round-2 GPU call BD: backward tail schedule under TN policy 7 (layers whose dW runs on the main stream)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02bd
mkdir -p $OUT
timeout -k 10 500 python -u scripts/step_ab.py --steps 20 --rounds 6 --settings default tail2 tail1 old_default tail2_ts1 > $OUT/step_ab.json 2> $OUT/step_ab.err; rc=$?; cat $OUT/step_ab.json; exit $rc
