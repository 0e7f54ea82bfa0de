set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_pair.py tests/test_gpu_full_step.py -q -x -p no:cacheprovider > gpurun_out/t_pair.log 2>&1; rc=$?
tail -30 gpurun_out/t_pair.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_full_bench.sh
