set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_rays.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/graph_tests.log 2>&1
rc=$?; echo "graph tests rc=$rc"; tail -5 $OUT/graph_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_full.py --steps 40 --warmup 5 > $OUT/bench_full.json 2> $OUT/bench_full.err && \
timeout -k 10 300 python scripts/bench_full.py --steps 40 --warmup 5 --graph > $OUT/bench_full_graph.json 2> $OUT/bench_full_graph.err && \
python -c "
import json
for f in ('bench_full', 'bench_full_graph'):
    d = json.load(open('$OUT/' + f + '.json')); print(f, round(d['value']), round(d['ms_per_step'], 3), d['losses']['loss'])"
