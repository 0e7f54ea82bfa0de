# round-2 GPU call AK: checkpoint validation -- all GPU tests, smoke, default bench, cfg3 (both modes), render
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02ak
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/tests.txt 2>&1; rc=$?; tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log && \
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err && echo "bench ok" && \
timeout -k 10 300 python scripts/bench_full.py --steps 40 --warmup 5 > $OUT/bench_full.json 2> $OUT/bench_full.err && echo "full ok" && \
timeout -k 10 300 python scripts/bench_render.py > $OUT/bench_render.json 2> $OUT/bench_render.err && echo "render ok" && \
timeout -k 10 300 python scripts/host_profile.py --plain > $OUT/host_cfg2.txt 2>&1 && tail -1 $OUT/host_cfg2.txt && \
timeout -k 10 300 python scripts/host_profile.py --plain --full > $OUT/host_cfg3.txt 2>&1 && tail -1 $OUT/host_cfg3.txt
