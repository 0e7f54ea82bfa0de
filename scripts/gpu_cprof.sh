set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m cProfile -s tottime scripts/bench_full.py --steps 40 --warmup 5 > gpurun_out/cprof_full.txt 2>&1 && head -80 gpurun_out/cprof_full.txt
