# PMC counters for the split-bf16 GEMMs (one launch per case, gemm_bench --quick --x6)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA -d $OUT/x6pmc1 -o run -- python $R/scripts/gemm_bench.py --quick --x6 > $OUT/x6pmc1.log 2>&1 && echo "pmc1 ok" && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_LDS_DATA_FIFO_FULL -d $OUT/x6pmc2 -o run -- python $R/scripts/gemm_bench.py --quick --x6 > $OUT/x6pmc2.log 2>&1 && echo "pmc2 ok"
