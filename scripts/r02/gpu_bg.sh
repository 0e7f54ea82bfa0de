# round-2 GPU call BG: l4's split count sized for its 64-wide skip segment (NERF_SEG2_SPLITS) A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02bg
mkdir -p $OUT
timeout -k 10 400 python -u scripts/step_ab.py --steps 20 --rounds 8 --settings default seg2_splits > $OUT/step_ab.json 2> $OUT/step_ab.err; rc=$?; cat $OUT/step_ab.json; [ $rc -eq 0 ] || exit $rc
NERF_SEG2_SPLITS=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_full_step.py > $OUT/tests.txt 2>&1; rc=$?; tail -1 $OUT/tests.txt; exit $rc
