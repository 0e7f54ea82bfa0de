# one GPU box call: parity tests, smoke, micro-benchmarks, bench, rocprofv3 kernel stats,
# HBM traffic counters (FETCH_SIZE / WRITE_SIZE in separate passes) of single GEMM launches
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -q -m gpu -p no:cacheprovider > $OUT/t_all.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -2 $OUT/t_all.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -m pytest tests/test_gpu_convergence.py -q -s -p no:cacheprovider > $OUT/psnr_parity.log 2>&1 && echo "psnr parity ok" && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && echo "smoke ok" && \
timeout -k 10 300 python scripts/gemm_bench.py --prec > $OUT/gemm_prec.txt 2>&1 && echo "gemm bench ok" && \
timeout -k 10 300 python scripts/composite_bench.py > $OUT/composite_bench.txt 2>&1 && echo "composite bench ok" && \
timeout -k 10 600 python bench.py --steps ${STEPS:-30} --warmup 5 > $OUT/bench.json 2> $OUT/bench.err && \
echo "bench ok" && \
timeout -k 10 300 python scripts/bench_render.py > $OUT/bench_render.json 2> $OUT/bench_render.err && \
echo "render bench ok" && \
timeout -k 10 300 python scripts/bench_full.py --steps 40 --warmup 5 > $OUT/bench_full.json 2> $OUT/bench_full.err && \
echo "full-step bench ok" && \
timeout -k 10 200 python scripts/gemm_bench.py --h16 --stamps > $OUT/stamps.txt 2>&1 && echo "stamps ok" && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt > $OUT/prof_bench.json 2> $OUT/prof.err && \
echo "prof ok" && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_full -o run -- python $R/scripts/bench_full.py --steps 10 --warmup 3 > $OUT/prof_full.json 2> $OUT/prof_full.err && \
echo "prof full ok" && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run -- python $R/scripts/gemm_bench.py --quick --h16 > $OUT/pmc_fetch.log 2>&1 && \
echo "pmc fetch ok" && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d $OUT/pmc_write -o run -- python $R/scripts/gemm_bench.py --quick --h16 > $OUT/pmc_write.log 2>&1 && \
echo "pmc write ok" && \
timeout -k 10 200 python $R/scripts/chain_bench.py > $OUT/chain_bench.txt 2>&1 && echo "chain bench ok" && \
(cd $R/scripts && timeout -k 10 300 python dw_bench.py --h16 > $OUT/dw_bench_h16.txt 2>&1) && echo "dw bench ok"
