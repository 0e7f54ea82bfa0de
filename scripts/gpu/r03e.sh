# round-3 GPU call E: the two-waves-per-SIMD chain kernels -- k_render_fused2 (eval) and
# k_mlp_chain_train2 (training forward): chain / frame / field-gradient tests, fused-eval
# ms/frame A/B against the one-wave kernel (NERF_FUSED_V1=1), training chain vs per-layer
# forward and cfg2 step A/B, the frame bench, kernel-trace stats and write-bytes PMC
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03e
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_field_grads.py "tests/test_gpu_distributed.py::test_full_frame_render_sharded_under_process_group_is_bit_identical" "tests/test_gpu_distributed.py::test_full_frame_render_matches_oracle_on_ray_subset" -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests.txt 2>&1; rc=$?; tail -8 $OUT/tests.txt; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u scripts/chain_bench.py --fused > $OUT/fused2.txt 2>&1 && cat $OUT/fused2.txt && \
NERF_FUSED_V1=1 timeout -k 10 200 python -u scripts/chain_bench.py --fused > $OUT/fused1.txt 2>&1 && cat $OUT/fused1.txt && \
timeout -k 10 200 python -u scripts/chain_bench.py > $OUT/chain_bench.txt 2>&1 && cat $OUT/chain_bench.txt && \
timeout -k 10 300 python -u scripts/step_ab.py --settings per_layer chain --rounds 4 > $OUT/step_ab_chain.json 2>&1 && cat $OUT/step_ab_chain.json && \
timeout -k 10 300 python -u scripts/bench_render.py --frames 5 --warmup 2 > $OUT/bench_render.json 2> $OUT/bench_render.err && cat $OUT/bench_render.json || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 $R/scripts/bench_render.py --frames 3 --warmup 1 > $OUT/prof.log 2>&1 && echo "prof ok" && \
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d $OUT/pmc_write -o run -- python3 $R/scripts/bench_render.py --frames 2 --warmup 1 > $OUT/pmc_write.log 2>&1 && echo "pmc write ok"
