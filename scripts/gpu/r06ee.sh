# round 6: the training forward chain's ReLU words swizzled per row (the 16 rows of a wave's
# LDS atomics on distinct banks): chain / render tests through the variant, its LDS counters,
# then the A/B against the tree
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=gpurun_out/r06ee; mkdir -p $O
NERF_HIP_LIB=$R/my-nope-nerf_amd/lib/ab/rswz.so timeout -k 10 500 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_render.py tests/test_gpu_native_bwd.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/rswz_tests.txt 2>&1 || exit $?
tail -1 $O/rswz_tests.txt
BENCH="$R/bench.py --steps 3 --warmup 2 --no-alt --no-cpu-baseline --no-cfg3 --exec eager"
(cd /tmp && export TMPDIR=/tmp NERF_HIP_LIB=$R/my-nope-nerf_amd/lib/ab/rswz.so && timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex k_mlp_chain_train2 --pmc SQ_WAVES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY -d $R/$O/pmc_rswz -o run -- python3 $BENCH > $R/$O/pmc_rswz.log 2>&1) || exit $?
echo "pmc ok"
(cd scripts && timeout -k 10 900 python -u lib_ab.py --rounds 3 --steps 30 my-nope-nerf_amd/lib/ab/rswz.so > ../$O/rswz_ab.txt 2>&1) || exit $?
grep median $O/rswz_ab.txt
