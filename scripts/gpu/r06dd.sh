# round 6: the weight-gradient operand images with swizzled column chunks (swz: the load waves'
# ds_write_b128 groups on distinct banks) -- job-list / weight-gradient tests through the variant,
# the A/B against the tree, and the variant's SQ LDS counters
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=gpurun_out/r06dd; mkdir -p $O
NERF_HIP_LIB=$R/my-nope-nerf_amd/lib/ab/swz.so timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_native_bwd.py tests/test_gpu_full_step.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "wgrad or weight or native or full" > $O/swz_tests.txt 2>&1 || exit $?
tail -1 $O/swz_tests.txt
BENCH="$R/bench.py --steps 3 --warmup 2 --no-alt --no-cpu-baseline --no-cfg3 --exec eager"
(cd /tmp && export TMPDIR=/tmp NERF_HIP_LIB=$R/my-nope-nerf_amd/lib/ab/swz.so && timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex k_wgrad_jobs --pmc SQ_WAVES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d $R/$O/pmc_swz -o run -- python3 $BENCH > $R/$O/pmc_swz.log 2>&1) || exit $?
echo "pmc ok"
(cd scripts && timeout -k 10 900 python -u lib_ab.py --rounds 3 --steps 30 my-nope-nerf_amd/lib/ab/swz.so > ../$O/swz_ab.txt 2>&1) || exit $?
grep median $O/swz_ab.txt
