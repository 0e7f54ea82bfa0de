# round-3 GPU call A: the whole GPU suite on the new tree (ABI 9, f16x3 default, in-place
# all-reduce, cfg4/cfg5 process-group tests), smoke, a short cfg2 bench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03a
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/tests.txt 2>&1; rc=$?; tail -15 $OUT/tests.txt; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --cpu-budget 10 > $OUT/bench.json 2> $OUT/bench.err && echo "bench ok" && cat $OUT/bench.json | head -c 600
