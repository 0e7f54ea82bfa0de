# fused layer chain bring-up: its parity tests first, then the bench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/chain_tests.log 2>&1
rc=$?; echo "chain tests rc=$rc"; tail -15 $OUT/chain_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-alt > $OUT/bench_chain.json 2> $OUT/bench_chain.err && \
python -c "import json; d=json.load(open('$OUT/bench_chain.json')); print('bench', round(d['value']), round(d['ms_per_step'],3))"
