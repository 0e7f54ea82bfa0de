# round-3 GPU call ZJ: closing check of the final tree -- full GPU suite, smoke, default bench, kernel stats
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03zj
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.txt 2>&1; rc=$?; tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log && \
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err && echo "bench ok" && python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'], d['ms_per_step'], d['ms_per_step_median'], d['execution'], d['roofline']['frac'], d['render_cfg4']['ms_per_frame'], d['render_cfg4']['roofline']['frac'])" || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_bench -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt --exec eager > $OUT/prof_bench.log 2>&1 && echo "prof bench ok"
