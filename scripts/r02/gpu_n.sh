# round-2 GPU call N: 4x4-chain HIP backwards -- ray/pose tests, full-step parity, graph tests, cfg3 bench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02n
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_rays.py tests/test_gpu_full_step.py tests/test_gpu_graph.py tests/test_gpu_dropin.py > $OUT/tests.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $OUT/tests.log | tail -15; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_full.py --steps 40 --warmup 5 > $OUT/bench_full_graph.json 2> $OUT/bench_full_graph.err && cat $OUT/bench_full_graph.json && \
timeout -k 10 300 python scripts/bench_full.py --steps 40 --warmup 5 --eager > $OUT/bench_full_eager.json 2> $OUT/bench_full_eager.err && cat $OUT/bench_full_eager.json && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr3g -o run -- python3 $R/scripts/bench_full.py --steps 12 --warmup 3 > $OUT/b3g.json 2> $OUT/b3g.err && echo "trace ok"
