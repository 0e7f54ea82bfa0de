# round-2 GPU call E: fused-eval parity, the plateau PSNR convergence study
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02e
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread \
  tests/test_gpu_chain.py > $OUT/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "FAILED|passed|failed|Error" $OUT/tests.log | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 1050 python -u scripts/convergence.py --steps 2000 > $OUT/convergence.jsonl 2> $OUT/convergence.log
echo "convergence rc=$?"
tail -1 $OUT/convergence.jsonl
