set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out
mkdir -p $OUT
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_INSTS_MFMA -d $OUT/pmc1 -o run -- python $R/scripts/gemm_bench.py --quick > $OUT/pmc1.log 2>&1
echo "pmc1 rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $OUT/pmc2 -o run -- python $R/scripts/gemm_bench.py --quick > $OUT/pmc2.log 2>&1
echo "pmc2 rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d $OUT/pmc3 -o run -- python $R/scripts/gemm_bench.py --quick > $OUT/pmc3.log 2>&1
echo "pmc3 rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d $OUT/pmc4 -o run -- python $R/scripts/gemm_bench.py --quick > $OUT/pmc4.log 2>&1
echo "pmc4 rc=$?"
