set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_rays.py tests/test_gpu_render.py tests/test_gpu_kernels.py -q -x -p no:cacheprovider > gpurun_out/t_rays.log 2>&1; rc=$?
tail -30 gpurun_out/t_rays.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-alt > gpurun_out/bench_rays.json 2> gpurun_out/bench_rays.err && cat gpurun_out/bench_rays.json
