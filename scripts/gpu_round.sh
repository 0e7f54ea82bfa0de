# one GPU box call: parity tests, smoke, micro-benchmarks, bench, rocprofv3 kernel stats
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -q -m gpu -p no:cacheprovider > $OUT/t_all.log 2>&1
echo "tests rc=$?"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && echo "smoke ok" && \
timeout -k 10 300 python scripts/gemm_bench.py > $OUT/gemm_bench.txt 2>&1 && echo "gemm bench ok" && \
timeout -k 10 300 python scripts/composite_bench.py > $OUT/composite_bench.txt 2>&1 && echo "composite bench ok" && \
timeout -k 10 600 python bench.py --steps ${STEPS:-30} --warmup 5 > $OUT/bench.json 2> $OUT/bench.err && \
echo "bench ok" && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.err && \
echo "prof ok"
