# round-3 GPU call G: training chain with the save work spread over the MFMA tiles: chain
# tests, forward A/B with ablations, cfg2 step A/B (per-layer forward vs the chain)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03g
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_field_grads.py -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests.txt 2>&1; rc=$?; tail -4 $OUT/tests.txt; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for lib in libnerf_hip ab/tr1 ab/tr2 ab/tr3; do
  NERF_HIP_LIB=$R/my-nope-nerf_amd/lib/$lib.so timeout -k 10 120 python -u scripts/chain_bench.py > $OUT/chain_$(basename $lib).txt 2>&1 || exit 3
  echo "$lib"; grep "keep=True: forward" $OUT/chain_$(basename $lib).txt
done
timeout -k 10 300 python -u scripts/step_ab.py --settings per_layer chain --rounds 4 > $OUT/step_ab_chain.json 2>&1 && cat $OUT/step_ab_chain.json
