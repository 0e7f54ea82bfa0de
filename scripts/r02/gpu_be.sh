# round-2 GPU call BE: chunk-per-block dyr kernel (heads backward mode 1) -- parity, kernel stats, step time
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02be
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_full_step.py tests/test_gpu_chain.py > $OUT/tests.txt 2>&1; rc=$?; tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/step_ab.py --steps 20 --rounds 6 --settings default tail3 > $OUT/step_ab.json 2> $OUT/step_ab.err; rc=$?; cat $OUT/step_ab.json; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt > $OUT/prof_bench.json 2> $OUT/prof.err && echo "prof ok" && grep -E "heads|Name" $OUT/prof/run_kernel_stats.csv | cut -c1-160
