# round-2 GPU call AC: parity of the LDS-staged epilogue operands; NT phase diagnostics (ablation, stamps)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02ac
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/tests.txt 2>&1; rc=$?; tail -3 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/nt_bench.py --ablate 0 > $OUT/nt.txt 2>/dev/null && \
timeout -k 10 300 python scripts/nt_bench.py --ablate 1 >> $OUT/nt.txt 2>/dev/null && \
timeout -k 10 300 python scripts/nt_bench.py --stamps >> $OUT/nt.txt 2>/dev/null && cat $OUT/nt.txt
