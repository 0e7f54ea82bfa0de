# round-3 GPU call ZH: the TN x tile as 4-row quarter strips on every thread (balanced waves):
# tests, phase stamps, standalone timings and the cfg2 step, libraries alternated (q0 = before)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03zh
mkdir -p $OUT
L=$R/my-nope-nerf_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_native_bwd.py tests/test_gpu_full_step.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests.txt 2>&1; rc=$?; tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
NERF_HIP_LIB=$L/ab/tstq.so timeout -k 10 100 python -u scripts/tn_stamps.py 2>/dev/null | tail -1
for r in 1 2; do for v in q0 new; do
  lib=$L/libnerf_hip.so; [ $v = new ] || lib=$L/ab/$v.so
  echo "$v tn round $r: $(NERF_HIP_LIB=$lib timeout -k 10 100 python -u scripts/tn_ablation.py 2> /dev/null | tail -1)"
done; done
for r in 1 2 3; do for v in q0 new; do
  lib=$L/libnerf_hip.so; [ $v = new ] || lib=$L/ab/$v.so
  NERF_HIP_LIB=$lib timeout -k 10 150 python -u scripts/step_ab.py --steps 20 --rounds 3 --settings default > $OUT/step_${v}_$r.txt 2>&1 || exit 4
  echo "$v step round $r: $(grep -o '"ms_per_step_median": [0-9.]*' $OUT/step_${v}_$r.txt)"
done; done
