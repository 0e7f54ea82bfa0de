# round-2 GPU call S: coalesced encode, single pack launch, deferred depth-prior affine -- parity + benches
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02s
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_full_step.py tests/test_gpu_graph.py tests/test_gpu_render.py tests/test_gpu_chain.py > $OUT/tests.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $OUT/tests.log | tail -15; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_full.py --steps 40 --warmup 5 > $OUT/bench_full_graph.json 2> $OUT/bench_full_graph.err && cat $OUT/bench_full_graph.json && \
timeout -k 10 300 python scripts/bench_full.py --steps 40 --warmup 5 --eager > $OUT/bench_full_eager.json 2> $OUT/bench_full_eager.err && cat $OUT/bench_full_eager.json && \
timeout -k 10 300 python -u scripts/step_ab.py --steps 20 --rounds 3 --settings default > $OUT/step.json 2> $OUT/step.err && tail -1 $OUT/step.json && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr2 -o run -- python3 $R/bench.py --steps 12 --warmup 3 --no-alt --no-cpu-baseline > $OUT/b2.json 2> $OUT/b2.err && echo "trace ok"
