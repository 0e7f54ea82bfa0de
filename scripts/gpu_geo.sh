set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_geometry.py -q -x -p no:cacheprovider > gpurun_out/t_geo.log 2>&1; rc=$?
tail -40 gpurun_out/t_geo.log
exit $rc
