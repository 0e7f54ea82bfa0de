# round-2 GPU call BC: TN policy 8 (eight-wave 128-output tiles) and the tail schedule under policy 7
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02bc
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "bwd_weight" > $OUT/tests_dw.txt 2>&1; rc=$?; tail -2 $OUT/tests_dw.txt; [ $rc -eq 0 ] || exit $rc
(cd scripts && timeout -k 10 200 python -u dw_policy_bench.py > $OUT/dw_policy.txt 2>&1); rc=$?; cat $OUT/dw_policy.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/step_ab.py --steps 20 --rounds 6 --settings default tn_narrow8 tail2 tail4 > $OUT/step_ab.json 2> $OUT/step_ab.err; rc=$?; cat $OUT/step_ab.json; exit $rc
