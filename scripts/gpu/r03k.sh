# round-3 GPU call K: save pieces de-phased across the two waves of a SIMD (training chain),
# packed-f32 epilogue unscale (both chain kernels): chain tests, forward A/B + stamps against
# the in-phase build, cfg2 step A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03k
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_field_grads.py -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests.txt 2>&1; rc=$?; tail -4 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
for lib in libnerf_hip ab/nodephase libnerf_hip ab/nodephase; do
  NERF_HIP_LIB=$R/my-nope-nerf_amd/lib/$lib.so timeout -k 10 120 python -u scripts/chain_bench.py > $OUT/chain_$(basename $lib).txt 2>&1 || exit 3
  echo "$lib"; grep "keep=True" $OUT/chain_$(basename $lib).txt
done
timeout -k 10 300 python -u scripts/step_ab.py --settings per_layer chain --rounds 4 > $OUT/step_ab_chain.json 2>&1 && cat $OUT/step_ab_chain.json
