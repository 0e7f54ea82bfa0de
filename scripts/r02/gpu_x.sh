# round-2 GPU call X: output heads fused into the l7 / colour-layer epilogues -- parity + step
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02x
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_render.py tests/test_gpu_full_step.py tests/test_golden.py tests/test_gpu_convergence.py > $OUT/tests.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $OUT/tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/step_ab.py --steps 20 --rounds 5 --settings default > $OUT/step.json 2> $OUT/step.err && tail -1 $OUT/step.json && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr2 -o run -- python3 $R/bench.py --steps 12 --warmup 3 --no-alt --no-cpu-baseline > $OUT/b2.json 2> $OUT/b2.err && echo "trace ok"
