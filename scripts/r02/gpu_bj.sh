# round-2 GPU call BJ: clean-rebuilt library -- kernel tests, smoke, default bench line
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02bj
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_render.py > $OUT/tests.txt 2>&1; rc=$?; tail -1 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log && \
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err && python -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['execution'], d['roofline']['frac'])"
