# round-3 GPU call ZL: last sanity check of the committed tree after the final rebuild (smoke + kernel / native-backward tests)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03zl
mkdir -p $OUT
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_native_bwd.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests.txt 2>&1; rc=$?; tail -2 $OUT/tests.txt; exit $rc
