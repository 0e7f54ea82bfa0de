# round-3 GPU call L: the next layer's A fragments split just in time inside the k-steps (one
# k-step ahead, between MFMA tiles) instead of all in the epilogue, both chain kernels: tests,
# A/B against the epilogue-split build (training forward, eval frame) and against column maxima
# taken from the stored values (training), cfg2 step A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03l
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_field_grads.py -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests.txt 2>&1; rc=$?; tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
NERF_HIP_LIB=$R/my-nope-nerf_amd/lib/ab/savefused.so timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -q -m gpu -k "chain_matches or gradients" --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests_savefused.txt 2>&1; rc=$?; tail -2 $OUT/tests_savefused.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for lib in libnerf_hip ab/nojit ab/savefused; do
  NERF_HIP_LIB=$R/my-nope-nerf_amd/lib/$lib.so timeout -k 10 120 python -u scripts/chain_bench.py > $OUT/chain_$(basename $lib)_$rep.txt 2>&1 || exit 3
  echo "$lib"; grep "keep=True" $OUT/chain_$(basename $lib)_$rep.txt
done
for lib in libnerf_hip ab/nojit; do
  NERF_HIP_LIB=$R/my-nope-nerf_amd/lib/$lib.so timeout -k 10 120 python -u scripts/chain_bench.py --fused > $OUT/fused_$(basename $lib)_$rep.txt 2>&1 || exit 3
  echo "$lib"; grep "fused eval" $OUT/fused_$(basename $lib)_$rep.txt
done
done
timeout -k 10 300 python -u scripts/step_ab.py --settings per_layer chain --rounds 4 > $OUT/step_ab_chain.json 2>&1 && cat $OUT/step_ab_chain.json
