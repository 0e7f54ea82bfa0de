# round-3 GPU call ZI: x sub-strips of 2 rows for the 64-column TN tiles (l0, the encoding tiles
# of the two-segment launches): tests, standalone dW timings and the cfg2 step vs HEAD (q4)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03zi
mkdir -p $OUT
L=$R/my-nope-nerf_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_native_bwd.py tests/test_gpu_full_step.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests.txt 2>&1; rc=$?; tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
for v in q4 new; do
  lib=$L/libnerf_hip.so; [ $v = new ] || lib=$L/ab/$v.so
  NERF_HIP_LIB=$lib timeout -k 10 100 python -u scripts/dw_policy_bench.py 2>/dev/null | grep "policy 7" | sed "s/^/$v /"
done
for r in 1 2 3; do for v in q4 new; do
  lib=$L/libnerf_hip.so; [ $v = new ] || lib=$L/ab/$v.so
  NERF_HIP_LIB=$lib timeout -k 10 150 python -u scripts/step_ab.py --steps 20 --rounds 3 --settings default > $OUT/step_${v}_$r.txt 2>&1 || exit 4
  echo "$v step round $r: $(grep -o '"ms_per_step_median": [0-9.]*' $OUT/step_${v}_$r.txt)"
done; done
