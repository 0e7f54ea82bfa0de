# round-2 GPU call J: kernel traces (timeline) of the cfg2 bench step and the cfg3 step (graph + eager)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02j
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr2 -o run -- python3 $R/bench.py --steps 12 --warmup 3 --no-alt --no-cpu-baseline > $OUT/b2.json 2> $OUT/b2.err && echo "cfg2 ok" && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr3g -o run -- python3 $R/scripts/bench_full.py --steps 12 --warmup 3 > $OUT/b3g.json 2> $OUT/b3g.err && echo "cfg3 graph ok" && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr3e -o run -- python3 $R/scripts/bench_full.py --steps 12 --warmup 3 --eager > $OUT/b3e.json 2> $OUT/b3e.err && echo "cfg3 eager ok"
find $OUT -name "*.csv" | head
