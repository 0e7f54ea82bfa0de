# round-2 GPU call AZ: eight-wave XCD-paired weight-gradient tiles (TN policy 7) -- parity, standalone, step A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02az
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "bwd_weight" > $OUT/tests_dw.txt 2>&1; rc=$?; tail -2 $OUT/tests_dw.txt; [ $rc -eq 0 ] || exit $rc
(cd scripts && timeout -k 10 200 python -u dw_policy_bench.py > $OUT/dw_policy.txt 2>&1); rc=$?; cat $OUT/dw_policy.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/step_ab.py --steps 20 --rounds 6 --settings tn3 tn_pair tn_pair8 > $OUT/step_ab.json 2> $OUT/step_ab.err; rc=$?; cat $OUT/step_ab.json; exit $rc
