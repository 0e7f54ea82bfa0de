# round-3 GPU call X: NT epilogue with packed-f32 unscale (float scales staged in LDS) and the
# ReLU mask as a sign-extended AND: kernel tests, standalone NT timings and the cfg2 step,
# libraries alternated (old = the previous commit)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03x
mkdir -p $OUT
L=$R/my-nope-nerf_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_chain.py tests/test_gpu_full_step.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests.txt 2>&1; rc=$?; tail -3 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for v in old new; do
  lib=$L/libnerf_hip.so; [ $v = new ] || lib=$L/ab/$v.so
  NERF_HIP_LIB=$lib timeout -k 10 100 python -u scripts/nt_bench.py --iters 30 > $OUT/nt_${v}_$r.json 2> $OUT/nt_${v}_$r.err || exit 3
  echo "$v nt round $r: $(cat $OUT/nt_${v}_$r.json)"
done; done
for r in 1 2; do for v in old new; do
  lib=$L/libnerf_hip.so; [ $v = new ] || lib=$L/ab/$v.so
  NERF_HIP_LIB=$lib timeout -k 10 150 python -u scripts/step_ab.py --steps 20 --rounds 3 --settings default > $OUT/step_${v}_$r.txt 2>&1 || exit 4
  echo "$v step round $r: $(grep -o '"ms_per_step_median": [0-9.]*' $OUT/step_${v}_$r.txt)"
done; done
