# round-3 GPU call V: the l1 + l0 tail weight gradients in one launch (native backward)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03v
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_native_bwd.py tests/test_gpu_full_step.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests.txt 2>&1; rc=$?; tail -3 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/step_ab.py --steps 20 --rounds 5 --settings default tail_two python_bwd > $OUT/step_ab.txt 2>&1 && tail -1 $OUT/step_ab.txt || exit 3
