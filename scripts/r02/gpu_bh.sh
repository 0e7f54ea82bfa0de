# round-2 GPU call BH: backward side-stream schedule variants under the final dW tiles
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02bh
mkdir -p $OUT
timeout -k 10 500 python -u scripts/step_ab.py --steps 20 --rounds 8 --settings default tail2_ts1 side2_tail2 tail2_ts2 > $OUT/step_ab.json 2> $OUT/step_ab.err; rc=$?; cat $OUT/step_ab.json; exit $rc
