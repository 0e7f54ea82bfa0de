set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python scripts/bench_full.py --steps 40 --warmup 5 > gpurun_out/bench_full_h.json 2>&1 && cat gpurun_out/bench_full_h.json
