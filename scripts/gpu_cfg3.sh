set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_render.py tests/test_gpu_pair.py tests/test_gpu_full_step.py -q -x -p no:cacheprovider > gpurun_out/t_cfg3.log 2>&1; rc=$?
tail -5 gpurun_out/t_cfg3.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_full.py --steps 40 --warmup 5 > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err && cat gpurun_out/bench_full.json && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-alt --no-cpu-baseline > gpurun_out/bench_q3.json 2>gpurun_out/bench_q3.err && \
python -c "
import json
d=json.load(open('gpurun_out/bench_q3.json')); print('cfg2', round(d['value']), round(d['ms_per_step'],3))"
