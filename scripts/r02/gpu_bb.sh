# round-2 GPU call BB: default TN policy 7 -- whole GPU suite, smoke, bench (cfg2), cfg3 bench, rocprof stats, PMC passes
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02bb
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.txt 2>&1; rc=$?; tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log && \
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err && echo "bench ok" && \
timeout -k 10 300 python scripts/bench_full.py --steps 40 --warmup 5 > $OUT/bench_full.json 2> $OUT/bench_full.err && echo "full ok" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt > $OUT/prof_bench.json 2> $OUT/prof.err && echo "prof ok" && \
BENCH="python3 $R/bench.py --steps 3 --warmup 2 --no-alt --no-cpu-baseline --exec eager" && REGEX='k_gemm_(nt|tn)_x6' && \
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE --kernel-include-regex "$REGEX" -d $OUT/pmc_fetch -o run -- $BENCH > $OUT/pmc_fetch.log 2>&1 && echo "pmc fetch ok" && \
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE --kernel-include-regex "$REGEX" -d $OUT/pmc_write -o run -- $BENCH > $OUT/pmc_write.log 2>&1 && echo "pmc write ok" && \
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "$REGEX" -d $OUT/pmc_sq -o run -- $BENCH > $OUT/pmc_sq.log 2>&1 && echo "pmc sq ok"
