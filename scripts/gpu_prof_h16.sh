set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python scripts/gemm_bench.py --prec > $OUT/gemm_prec.txt 2>&1 && echo "gemm bench ok" && \
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --gemm-precision f16x3 --no-cpu-baseline --no-alt > $OUT/bench_h16.json 2> $OUT/bench_h16.err && \
echo "bench ok" && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_h16 -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt > $OUT/prof_h16.json 2> $OUT/prof_h16.err && \
echo "prof ok"
