# round-2 GPU call AY: write-through (sc1) GEMM output / slab stores -- step A/B, parity under NERF_STORE_NT=2
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02ay
mkdir -p $OUT
timeout -k 10 400 python -u scripts/step_ab.py --steps 20 --rounds 6 --settings default store_sc1 > $OUT/step_ab.json 2> $OUT/step_ab.err; rc=$?; cat $OUT/step_ab.json; [ $rc -eq 0 ] || exit $rc
NERF_STORE_NT=2 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_full_step.py tests/test_gpu_render.py > $OUT/tests_sc1.txt 2>&1; rc=$?; tail -2 $OUT/tests_sc1.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/step_ab.py --steps 20 --rounds 6 --settings store_sc1 default > $OUT/step_ab2.json 2> $OUT/step_ab2.err; rc=$?; cat $OUT/step_ab2.json; exit $rc
