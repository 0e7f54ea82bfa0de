# split-bf16 GEMM: parity tests (both precisions), phase stamps, GEMM A/B, bench in both modes
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -q -m gpu -p no:cacheprovider -x > $OUT/t_all.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -3 $OUT/t_all.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python scripts/gemm_bench.py --x6 --stamps > $OUT/stamps.txt 2>&1 && echo "stamps ok" && \
timeout -k 10 300 python scripts/gemm_bench.py --prec > $OUT/gemm_prec.txt 2>&1 && echo "gemm bench ok" && \
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --gemm-precision bf16x6 > $OUT/bench_x6.json 2> $OUT/bench_x6.err && echo "bench x6 ok"
