# round-3 GPU call C: exact-f32 NT with the operand-swapped float4 epilogue (kernel tests in
# every mode, per-kind times, clock / MFMA-busy PMC pass), fused-eval phase stamps, bench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03c
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_render.py -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests.txt 2>&1; rc=$?; tail -4 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/gemm_bench.py --prec > $OUT/gemm_prec.txt 2>&1 && cat $OUT/gemm_prec.txt
timeout -k 10 120 python -u scripts/f32_clock.py > $OUT/f32_clock.json 2>&1 && cat $OUT/f32_clock.json
timeout -k 10 200 python -u scripts/chain_bench.py --fused > $OUT/fused_phases.txt 2>&1 && cat $OUT/fused_phases.txt
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err && echo "bench ok" && head -c 900 $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES -d $OUT/pmc_f32 -o run -- python3 $R/scripts/f32_clock.py --seconds 1 > $OUT/pmc_f32.log 2>&1 && echo "pmc f32 ok"
