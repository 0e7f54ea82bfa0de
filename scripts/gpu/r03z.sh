# round-3 GPU call Z: HIP gradients vs the oracle in fp64 next to the fp32 reference's own distance
# to fp64, plus the tightened pose / ray gradient bars (render + full-step tests)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03z
mkdir -p $OUT
rm -f $OUT/errs.jsonl
NERF_ERR_REPORT=$OUT/errs.jsonl timeout -k 10 500 python -u -m pytest tests/test_gpu_render.py tests/test_gpu_full_step.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.txt 2>&1; rc=$?; tail -8 $OUT/tests.txt; exit $rc
