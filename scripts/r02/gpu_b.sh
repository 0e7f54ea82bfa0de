# round-2 GPU call B: new parity tests first, then the whole GPU suite, smoke, bench, rocprof
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02b
mkdir -p $OUT
timeout -k 10 1500 python -u -m pytest -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_distributed.py tests/test_gpu_dropin.py tests/test_gpu_full_step.py tests/test_gpu_render.py \
  tests/test_golden.py tests > $OUT/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $OUT/tests.log | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && echo "smoke ok" && \
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err && echo "bench ok" && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt > $OUT/prof_bench.json 2> $OUT/prof.err && \
echo "prof ok"
