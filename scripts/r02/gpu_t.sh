# round-2 GPU call T: fused depth-prior affine -- parity + cfg3 benches
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02t
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_rays.py tests/test_gpu_full_step.py tests/test_gpu_graph.py > $OUT/tests.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $OUT/tests.log | tail -15; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_full.py --steps 40 --warmup 5 > $OUT/bench_full_graph.json 2> $OUT/bench_full_graph.err && cat $OUT/bench_full_graph.json && \
timeout -k 10 300 python scripts/bench_full.py --steps 40 --warmup 5 --eager > $OUT/bench_full_eager.json 2> $OUT/bench_full_eager.err && cat $OUT/bench_full_eager.json
