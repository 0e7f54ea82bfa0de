# round 6: the new default (epilogue row maxima by v_max3): GPU suite; then the forward chain's LDS
# bank conflicts (PMC: SQ_LDS_BANK_CONFLICT / ADDR_CONFLICT) in the default build against ReLU-word
# rows padded to 9 words (m9) and that plus 4 column-max copies (cm4m9), and their lib A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=gpurun_out/r06j; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1 || exit $?
tail -1 $O/tests.txt
NERF_HIP_LIB=$R/my-nope-nerf_amd/lib/ab/cm4m9.so timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/cm4m9_tests.txt 2>&1 || exit $?
tail -1 $O/cm4m9_tests.txt
BENCH="$R/bench.py --steps 3 --warmup 2 --no-alt --no-cpu-baseline --no-cfg3 --exec eager"
CT="SQ_WAVES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_WAVE_CYCLES SQ_WAIT_INST_LDS"
for v in default m9 cm4m9; do
  if [ $v = default ]; then LIB=$R/my-nope-nerf_amd/lib/libnerf_hip.so; else LIB=$R/my-nope-nerf_amd/lib/ab/$v.so; fi
  (cd /tmp && export TMPDIR=/tmp NERF_HIP_LIB=$LIB && timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex k_mlp_chain --pmc $CT -d $R/$O/pmc_lds_$v -o run -- python3 $BENCH > $R/$O/pmc_lds_$v.log 2>&1) || exit $?
  echo "pmc ok $v"
done
(cd scripts && timeout -k 10 1000 python -u lib_ab.py --rounds 3 --steps 20 my-nope-nerf_amd/lib/ab/m9.so my-nope-nerf_amd/lib/ab/cm4m9.so > ../$O/lds_ab.txt 2>&1) || exit $?
grep median $O/lds_ab.txt
