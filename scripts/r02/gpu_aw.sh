# round-2 GPU call AW: XCD-paired 256x128 weight-gradient tiles (TN policy 4) -- parity, step A/B, whole suite
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02aw
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "bwd_weight" > $OUT/tests_dw.txt 2>&1; rc=$?; tail -2 $OUT/tests_dw.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/step_ab.py --steps 20 --rounds 5 --settings tn3 tn_pair > $OUT/step_ab.json 2> $OUT/step_ab.err; rc=$?; cat $OUT/step_ab.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.txt 2>&1; rc=$?; tail -3 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log
