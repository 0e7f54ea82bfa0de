set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -q -m gpu -p no:cacheprovider > $OUT/t_all.log 2>&1
echo "tests rc=$?"
timeout -k 10 300 python scripts/gemm_bench.py > $OUT/gemm_bench.txt 2>&1 && echo "gemm bench ok" && \
timeout -k 10 600 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err && echo "bench ok"
