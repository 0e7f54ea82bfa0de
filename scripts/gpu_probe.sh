set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -m gpu -p no:cacheprovider -k "adam" > $OUT/t_adam.log 2>&1
echo "adam test rc=$?"
timeout -k 10 300 python scripts/graph_probe.py > $OUT/graph_probe.log 2>&1
echo "probe rc=$?"
