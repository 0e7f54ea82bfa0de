# round-2 GPU call AA: bias / v staged in LDS for the fp16-pair NT epilogue -- GEMM parity, then bench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02aa
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_full_step.py > $OUT/tests.txt 2>&1 && tail -2 $OUT/tests.txt && \
timeout -k 10 300 python scripts/nt_bench.py > $OUT/nt_bench.txt 2>&1 && cat $OUT/nt_bench.txt | tail -12 && \
timeout -k 10 600 python bench.py --no-alt --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err && echo bench ok && \
timeout -k 10 300 python scripts/bench_full.py --steps 40 --warmup 5 --mode eager > $OUT/bench_full.json 2> $OUT/bench_full.err && echo full ok
