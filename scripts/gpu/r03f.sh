# round-3 GPU call F: the chain kernels after the head-weight load fix (chain / frame tests),
# training-chain ablations (diagnostic libraries: no activation stores / no ReLU words and
# column maxima / neither / nothing stored), fused eval ms/frame
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03f
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_field_grads.py "tests/test_gpu_distributed.py::test_full_frame_render_sharded_under_process_group_is_bit_identical" "tests/test_gpu_distributed.py::test_full_frame_render_matches_oracle_on_ray_subset" -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests.txt 2>&1; rc=$?; tail -8 $OUT/tests.txt; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for lib in libnerf_hip ab/tr1 ab/tr2 ab/tr3 ab/tr7; do
  NERF_HIP_LIB=$R/my-nope-nerf_amd/lib/$lib.so timeout -k 10 120 python -u scripts/chain_bench.py > $OUT/chain_$(basename $lib).txt 2>&1 || exit 3
  echo "$lib"; grep "keep=True: forward" $OUT/chain_$(basename $lib).txt
done
timeout -k 10 200 python -u scripts/chain_bench.py --fused > $OUT/fused2.txt 2>&1 && cat $OUT/fused2.txt
