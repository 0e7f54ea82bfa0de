# round-2 GPU call G: store-hint A/B; PMC passes (HBM bytes, SQ cycles) of the in-step NT / TN GEMMs
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02g
mkdir -p $OUT
timeout -k 10 300 python -u scripts/step_ab.py --steps 20 --rounds 3 --settings default store_nt > $OUT/step_ab.json 2> $OUT/step_ab.err && echo "ab ok" && cat $OUT/step_ab.json
cd /tmp && export TMPDIR=/tmp
BENCH="python $R/bench.py --steps 3 --warmup 2 --no-alt --no-cpu-baseline"
REGEX='k_gemm_(nt|tn)_x6'
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE --kernel-include-regex "$REGEX" -d $OUT/pmc_fetch -o run -- $BENCH > $OUT/pmc_fetch.log 2>&1 && echo "pmc fetch ok" && \
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE --kernel-include-regex "$REGEX" -d $OUT/pmc_write -o run -- $BENCH > $OUT/pmc_write.log 2>&1 && echo "pmc write ok" && \
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "$REGEX" -d $OUT/pmc_sq -o run -- $BENCH > $OUT/pmc_sq.log 2>&1 && echo "pmc sq ok"
ls $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_sq 2>/dev/null | head
