set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06c; mkdir -p $O
L=$GRAFT_REPO_ROOT/my-nope-nerf_amd/lib/ab
NERF_HIP_LIB=$L/lag8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $O/lag8_chain_tests.txt 2>&1 || exit $?
tail -1 $O/lag8_chain_tests.txt
(cd scripts && timeout -k 10 900 python -u lib_ab.py --rounds 2 --steps 20 my-nope-nerf_amd/lib/ab/lag4.so my-nope-nerf_amd/lib/ab/lag8.so > ../$O/lag_ab.txt 2>&1) || exit $?
tail -3 $O/lag_ab.txt
NERF_HIP_LIB=$L/stamps.so timeout -k 10 300 python -u scripts/chain_bench.py > $O/stamps_train.txt 2>&1 || exit $?
NERF_HIP_LIB=$L/stamps.so timeout -k 10 300 python -u scripts/chain_bench.py --fused > $O/stamps_fused.txt 2>&1 || exit $?
tail -2 $O/stamps_train.txt; tail -1 $O/stamps_fused.txt
