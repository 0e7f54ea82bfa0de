# round-3 GPU call U: per-wave SQ cycle buckets of the standalone input-gradient NT and weight-
# gradient TN kernels (one PMC pass each, 8 SQ counters), to see what bounds them
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03u
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
C="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS"
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex 'k_gemm_nt_x6' --pmc $C -d $OUT/pmc_nt -o run -- python3 $R/scripts/nt_bench.py --iters 10 > $OUT/pmc_nt.log 2>&1 && echo "pmc nt ok" && \
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex 'k_gemm_tn_x6' --pmc $C -d $OUT/pmc_tn -o run -- python3 $R/scripts/dw_policy_bench.py > $OUT/pmc_tn.log 2>&1 && echo "pmc tn ok" && \
C2="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT" && \
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex 'k_gemm_nt_x6' --pmc $C2 -d $OUT/pmc_nt2 -o run -- python3 $R/scripts/nt_bench.py --iters 10 > $OUT/pmc_nt2.log 2>&1 && echo "pmc nt2 ok" && \
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex 'k_gemm_tn_x6' --pmc $C2 -d $OUT/pmc_tn2 -o run -- python3 $R/scripts/dw_policy_bench.py > $OUT/pmc_tn2.log 2>&1 && echo "pmc tn2 ok"
