# round-3 GPU call Y: survey of the observed gradient errors vs the oracle (render backward,
# ray gradients, the cfg3 full step in every GEMM mode) to set the tolerances from
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03y
mkdir -p $OUT
rm -f $OUT/errs.jsonl
NERF_ERR_REPORT=$OUT/errs.jsonl timeout -k 10 500 python -u -m pytest tests/test_gpu_render.py tests/test_gpu_full_step.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.txt 2>&1; rc=$?; tail -3 $OUT/tests.txt; wc -l $OUT/errs.jsonl; exit $rc
