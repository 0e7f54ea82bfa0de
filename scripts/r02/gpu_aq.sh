# round-2 GPU call AQ: final-tree kernel stats of the bench command and PMC passes (HBM bytes, SQ cycles)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02aq
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt > $OUT/prof_bench.json 2> $OUT/prof.err && echo "prof ok" && \
BENCH="python3 $R/bench.py --steps 3 --warmup 2 --no-alt --no-cpu-baseline --exec eager" && REGEX='k_gemm_(nt|tn)_x6' && \
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE --kernel-include-regex "$REGEX" -d $OUT/pmc_fetch -o run -- $BENCH > $OUT/pmc_fetch.log 2>&1 && echo "pmc fetch ok" && \
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE --kernel-include-regex "$REGEX" -d $OUT/pmc_write -o run -- $BENCH > $OUT/pmc_write.log 2>&1 && echo "pmc write ok" && \
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "$REGEX" -d $OUT/pmc_sq -o run -- $BENCH > $OUT/pmc_sq.log 2>&1 && echo "pmc sq ok"
