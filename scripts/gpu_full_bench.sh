set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python scripts/bench_full.py --steps 20 --warmup 5 > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err && cat gpurun_out/bench_full.json && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_full -o run -- python $R/scripts/bench_full.py --steps 10 --warmup 3 > $R/gpurun_out/prof_full.json 2> $R/gpurun_out/prof_full.err && echo prof ok
