# round 6: what the training chains wait on (PMC passes: vector-memory issue, LDS, instruction issue),
# the eval prologue's loads ahead of its DMAs (evpro), and the input-gradient chain's column maxima over 4 / 8 lanes into per-lane-group LDS copies (lib A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06f; mkdir -p $O
BENCH="$GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 --no-alt --no-cpu-baseline --no-cfg3 --exec eager"
pmc() {
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex k_mlp_chain --pmc $2 -d $GRAFT_REPO_ROOT/$O/pmc_$1 -o run -- python3 $BENCH > $GRAFT_REPO_ROOT/$O/pmc_$1.log 2>&1) || exit $?
  echo "pmc ok $1"
}
pmc vm "SQ_WAVES SQ_WAVE_CYCLES SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum"
pmc lds "SQ_WAVES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES"
pmc iss "SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_IFETCH SQ_BUSY_CYCLES SQ_INST_LEVEL_LDS"
pmc wt "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_MFMA"
NERF_HIP_LIB=$GRAFT_REPO_ROOT/my-nope-nerf_amd/lib/ab/evpro.so timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $O/evpro_tests.txt 2>&1 || exit $?
tail -1 $O/evpro_tests.txt
(cd scripts && timeout -k 10 1000 python -u lib_ab.py --rounds 2 --steps 20 my-nope-nerf_amd/lib/ab/cmqb4.so my-nope-nerf_amd/lib/ab/cmqb2.so my-nope-nerf_amd/lib/ab/evpro.so > ../$O/cmq_ab.txt 2>&1) || exit $?
grep median $O/cmq_ab.txt
