# round-2 GPU call AU: scalar where fallbacks + fused torch Adams in the cfg3 bench -- parity, cfg3 both modes x2
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02au
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_full_step.py tests/test_gpu_pair.py > $OUT/tests.txt 2>&1; rc=$?; tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python scripts/bench_full.py --steps 40 --warmup 5 > $OUT/full_$r.json 2> $OUT/full_$r.err || exit 1
  python -c "import json; f=json.load(open('$OUT/full_$r.json')); print({k:(round(v['ms_per_step'],3), round(v['host_ms_per_step_median'],3)) for k,v in f['runs'].items()})"
done
