set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -q -m gpu -p no:cacheprovider > gpurun_out/t_kernels.log 2>&1
rc=$?
echo "kernels rc=$rc"
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 600 python -m pytest tests/test_gpu_render.py -q -m gpu -p no:cacheprovider > gpurun_out/t_render.log 2>&1
  echo "render rc=$?"
fi
