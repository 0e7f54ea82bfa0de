# round-2 GPU call I (re-entry baseline): dW tiling / store-hint A/B on the step, cfg3 graph + eager, bench line
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02i
mkdir -p $OUT
timeout -k 10 400 python -u scripts/step_ab.py --steps 20 --rounds 3 > $OUT/step_ab.json 2> $OUT/step_ab.err && echo "ab ok" && cat $OUT/step_ab.json && \
timeout -k 10 300 python scripts/bench_full.py --steps 40 --warmup 5 > $OUT/bench_full_graph.json 2> $OUT/bench_full_graph.err && echo "full graph ok" && cat $OUT/bench_full_graph.json && \
timeout -k 10 300 python scripts/bench_full.py --steps 40 --warmup 5 --eager > $OUT/bench_full_eager.json 2> $OUT/bench_full_eager.err && echo "full eager ok" && cat $OUT/bench_full_eager.json && \
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err && echo "bench ok" && cat $OUT/bench.json
