# round-3 GPU call ZD: the TN main loop with two k-tiles per barrier (NERF_TN_PAIR build):
# weight-gradient tests with that library, standalone timings, the cfg2 step, libraries alternated
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03zd
mkdir -p $OUT
L=$R/my-nope-nerf_amd/lib
NERF_HIP_LIB=$L/ab/pair.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x -k "bwd_weight or split_accuracy_weight" --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests.txt 2>&1; rc=$?; tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for v in base pair; do
  lib=$L/libnerf_hip.so; [ $v = base ] || lib=$L/ab/$v.so
  echo "$v tn round $r: $(NERF_HIP_LIB=$lib timeout -k 10 100 python -u scripts/tn_ablation.py 2> /dev/null | tail -1)"
done; done
for r in 1 2; do for v in base pair; do
  lib=$L/libnerf_hip.so; [ $v = base ] || lib=$L/ab/$v.so
  NERF_HIP_LIB=$lib timeout -k 10 150 python -u scripts/step_ab.py --steps 20 --rounds 3 --settings default > $OUT/step_${v}_$r.txt 2>&1 || exit 4
  echo "$v step round $r: $(grep -o '"ms_per_step_median": [0-9.]*' $OUT/step_${v}_$r.txt)"
done; done
