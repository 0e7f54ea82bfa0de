# round-2 GPU call P: full GPU suite after the 4x4-chain / encode-backward changes
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02p
mkdir -p $OUT
timeout -k 10 1100 python -u -m pytest -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread tests > $OUT/tests.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $OUT/tests.log | tail -15; exit $rc
