set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_render.py -q -x -p no:cacheprovider > gpurun_out/t_direct.log 2>&1; rc=$?
tail -3 gpurun_out/t_direct.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/gemm_bench.py --x6 > gpurun_out/gb_direct.txt 2>&1 && \
NERF_NT_DIRECT=0 timeout -k 10 200 python scripts/gemm_bench.py --x6 > gpurun_out/gb_lds.txt 2>&1 && \
timeout -k 10 200 python scripts/gemm_bench.py --x6 --stamps > gpurun_out/stamps_direct.txt 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-alt --no-cpu-baseline > gpurun_out/bench_direct.json 2>gpurun_out/bench_direct.err && \
NERF_NT_DIRECT=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-alt --no-cpu-baseline > gpurun_out/bench_lds.json 2>gpurun_out/bench_lds.err && \
echo direct && cat gpurun_out/gb_direct.txt && echo lds && cat gpurun_out/gb_lds.txt && grep -h "cycles median" gpurun_out/stamps_direct.txt && \
python -c "
import json
for n in ('direct','lds'):
    d=json.load(open('gpurun_out/bench_%s.json'%n)); print(n, round(d['value']), round(d['ms_per_step'],3))"
