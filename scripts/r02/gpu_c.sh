# round-2 GPU call C: fused eval kernel parity + render bench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02c
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread \
  tests/test_gpu_chain.py tests/test_gpu_render.py tests/test_gpu_dropin.py > $OUT/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed|Error" $OUT/tests.log | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python scripts/bench_render.py --frames 10 > $OUT/bench_render.json 2> $OUT/bench_render.err && echo "render bench ok" && \
NERF_FUSED=0 timeout -k 10 300 python scripts/bench_render.py --frames 10 > $OUT/bench_render_unfused.json 2> $OUT/bench_render_unfused.err && echo "render bench unfused ok" && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python $R/scripts/bench_render.py --frames 5 > $OUT/prof_render.json 2> $OUT/prof.err && \
echo "prof ok"
cat $OUT/bench_render.json $OUT/bench_render_unfused.json
