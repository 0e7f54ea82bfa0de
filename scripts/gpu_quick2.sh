set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_render.py tests/test_gpu_rays.py -q -x -p no:cacheprovider > gpurun_out/t_q2.log 2>&1; rc=$?
tail -3 gpurun_out/t_q2.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-alt --no-cpu-baseline > gpurun_out/bench_q2.json 2>gpurun_out/bench_q2.err && \
python -c "
import json
d=json.load(open('gpurun_out/bench_q2.json')); print(round(d['value']), round(d['ms_per_step'],3))" && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof2 -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt > $GRAFT_REPO_ROOT/gpurun_out/prof2_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof2.err && echo prof ok
