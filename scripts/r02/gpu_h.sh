# round-2 GPU call H: graph tests, cfg3 bench (graph default + eager), bench line
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02h
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread \
  tests/test_gpu_graph.py tests/test_gpu_full_step.py > $OUT/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "FAILED|passed|failed|Error" $OUT/tests.log | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python scripts/bench_full.py --steps 40 --warmup 5 > $OUT/bench_full_graph.json 2> $OUT/bench_full_graph.err && echo "full graph ok" && cat $OUT/bench_full_graph.json
timeout -k 10 300 python scripts/bench_full.py --steps 40 --warmup 5 --eager > $OUT/bench_full_eager.json 2> $OUT/bench_full_eager.err && echo "full eager ok" && cat $OUT/bench_full_eager.json
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err && echo "bench ok" && cat $OUT/bench.json
