# round-2 GPU call W: 256x64 weight-gradient tile for the 64-wide inputs
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02w
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_render.py > $OUT/tests.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $OUT/tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/dw_bench.py --h16 > $OUT/dw.txt 2>&1 && grep default $OUT/dw.txt && \
timeout -k 10 300 python -u scripts/step_ab.py --steps 20 --rounds 5 --settings default > $OUT/step.json 2> $OUT/step.err && tail -1 $OUT/step.json
