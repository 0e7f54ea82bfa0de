# round 6: the gradient all-reduce on RCCL (world 1, the new test) and a probe of two RCCL ranks
# on the box's one GPU
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06u; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_distributed.py -m gpu -v -x --timeout 300 --timeout-method thread -p no:cacheprovider -k "rccl" > $O/rccl_tests.txt 2>&1 || exit $?
tail -4 $O/rccl_tests.txt
timeout -k 10 120 python -u scripts/probes/rccl_two_ranks.py > $O/rccl_two_ranks.txt 2>&1
echo "probe rc=$?"
grep -h '"rank"' $O/rccl_two_ranks.txt || tail -5 $O/rccl_two_ranks.txt
