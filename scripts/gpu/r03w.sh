# round-3 GPU call W: closing validation (native backward, two-segment dW) of the round's tree -- the full GPU suite, smoke, the
# default bench line, the frame render and cfg3 benches, kernel-trace stats of the bench and
# of the render
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03w
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests.txt 2>&1; rc=$?; tail -3 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log && \
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err && echo "bench ok" && head -c 700 $OUT/bench.json && echo && \
timeout -k 10 200 python -u scripts/bench_render.py --frames 5 --warmup 2 > $OUT/bench_render.json 2> $OUT/bench_render.err && cat $OUT/bench_render.json && \
timeout -k 10 300 python -u scripts/bench_full.py > $OUT/bench_full.json 2> $OUT/bench_full.err && head -c 600 $OUT/bench_full.json && echo || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_bench -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt --exec eager > $OUT/prof_bench.log 2>&1 && echo "prof bench ok" && \
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_render -o run -- python3 $R/scripts/bench_render.py --frames 3 --warmup 1 > $OUT/prof_render.log 2>&1 && echo "prof render ok"
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-alt --exec eager > $OUT/trace.log 2>&1 && echo "trace ok" && \
python3 $R/scripts/timeline.py $(ls $OUT/trace/*/run_kernel_trace.csv | head -1) > $OUT/timeline.txt 2>&1; echo timeline rc=$?
