# round-2 GPU call Z: checkpoint of the tree -- smoke, bench line, cfg3, render, kernel stats
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02z
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log && \
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err && echo "bench ok" && \
timeout -k 10 300 python scripts/bench_full.py --steps 40 --warmup 5 > $OUT/bench_full.json 2> $OUT/bench_full.err && echo "full ok" && \
timeout -k 10 300 python scripts/bench_render.py > $OUT/bench_render.json 2> $OUT/bench_render.err && echo "render ok" && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt > $OUT/prof_bench.json 2> $OUT/prof.err && echo "prof ok"
