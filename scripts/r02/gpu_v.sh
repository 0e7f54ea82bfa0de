# round-2 GPU call V: host-overhead cuts -- full GPU suite, cfg3 eager/graph, host profile, cfg2 bench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02v
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread tests > $OUT/tests.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $OUT/tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_full.py --steps 40 --warmup 5 --eager > $OUT/bench_full_eager.json 2> $OUT/bench_full_eager.err && cat $OUT/bench_full_eager.json && \
timeout -k 10 300 python scripts/bench_full.py --steps 40 --warmup 5 > $OUT/bench_full_graph.json 2> $OUT/bench_full_graph.err && cat $OUT/bench_full_graph.json && \
timeout -k 10 300 python -u scripts/host_profile.py --full > $OUT/host_full.txt 2> $OUT/host_full.err && head -1 $OUT/host_full.txt && \
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err && cat $OUT/bench.json
