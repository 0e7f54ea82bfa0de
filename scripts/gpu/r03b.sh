# round-3 GPU call B: the fixed process-group tests + fused-eval composite, NT main-loop /
# epilogue ablations (diagnostic libraries), exact-f32 clock PMC pass, cfg4 render + its
# write-bytes PMC pass
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03b
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest "tests/test_gpu_distributed.py::test_full_frame_render_sharded_under_process_group_is_bit_identical" "tests/test_gpu_distributed.py::test_full_frame_render_matches_oracle_on_ray_subset" tests/test_gpu_chain.py tests/test_gpu_field_grads.py "tests/test_gpu_kernels.py::test_pack_split_images" -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests.txt 2>&1; rc=$?; tail -6 $OUT/tests.txt; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for lib in libnerf_hip ab/nt2 ab/nt4 ab/nt8 ab/nt14 ab/epi8 ab/epi16 ab/epi24; do
  NERF_HIP_LIB=$R/my-nope-nerf_amd/lib/$lib.so timeout -k 10 120 python -u scripts/nt_bench.py --iters 30 > $OUT/nt_$(basename $lib).json 2>&1 || exit 3
  echo "$lib $(cat $OUT/nt_$(basename $lib).json | tail -1)"
done
timeout -k 10 120 python -u scripts/nt_bench.py --stamps > $OUT/nt_stamps.json 2>&1 && tail -2 $OUT/nt_stamps.json
timeout -k 10 120 python -u scripts/f32_clock.py > $OUT/f32_clock.json 2>&1 && cat $OUT/f32_clock.json
timeout -k 10 300 python -u scripts/bench_render.py --frames 5 --warmup 2 > $OUT/bench_render.json 2> $OUT/bench_render.err && cat $OUT/bench_render.json
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES -d $OUT/pmc_f32 -o run -- python3 $R/scripts/f32_clock.py --seconds 1 > $OUT/pmc_f32.log 2>&1 && echo "pmc f32 ok" && \
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d $OUT/pmc_write -o run -- python3 $R/scripts/bench_render.py --frames 2 --warmup 1 > $OUT/pmc_write.log 2>&1 && echo "pmc write ok" && \
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run -- python3 $R/scripts/bench_render.py --frames 2 --warmup 1 > $OUT/pmc_fetch.log 2>&1 && echo "pmc fetch ok"
