# fp16-pair GEMM checks: kernel parity first, then dW / GEMM A/B, bench, the full GPU suite
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/h16_kernels.log 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -3 $OUT/h16_kernels.log
[ $rc -eq 0 ] || exit $rc
(cd scripts && timeout -k 10 300 python dw_bench.py --h16 > $OUT/dw_bench_h16.txt 2>&1) && echo "dw bench ok" && \
timeout -k 10 300 python scripts/gemm_bench.py --prec > $OUT/gemm_prec.txt 2>&1 && echo "gemm bench ok" && \
timeout -k 10 600 python bench.py --steps 30 --warmup 5 --gemm-precision f16x3 --no-cpu-baseline > $OUT/bench_h16.json 2> $OUT/bench_h16.err && \
echo "bench ok" && \
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/t_all.log 2>&1
rc=$?; echo "all tests rc=$rc"; tail -5 $OUT/t_all.log
