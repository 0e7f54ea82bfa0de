# round-2 GPU call AP: host enqueue after the param-list / submodule caches; training-path parity
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02ap
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_full_step.py tests/test_gpu_graph.py tests/test_gpu_distributed.py > $OUT/tests.txt 2>&1; rc=$?; tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/host_profile.py --plain > $OUT/host_cfg2.txt 2>&1 && tail -1 $OUT/host_cfg2.txt && \
timeout -k 10 300 python scripts/host_profile.py --plain --full > $OUT/host_cfg3.txt 2>&1 && tail -1 $OUT/host_cfg3.txt && \
timeout -k 10 300 python scripts/host_profile.py --same-thread > $OUT/prof_cfg2.txt 2>&1 && head -2 $OUT/prof_cfg2.txt
