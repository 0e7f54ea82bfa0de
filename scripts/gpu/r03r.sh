# round-3 GPU call R: depth of the eight-wave TN operand pipeline (NERF_TN_NS 1 / 3 / 4):
# standalone weight-gradient timings per library, then the cfg2 step alternating libraries
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03r
mkdir -p $OUT
L=$R/my-nope-nerf_amd/lib
for v in base ns3 ns4; do
  lib=$L/libnerf_hip.so; [ $v = base ] || lib=$L/ab/$v.so
  NERF_HIP_LIB=$lib timeout -k 10 120 python -u scripts/dw_policy_bench.py > $OUT/dw_$v.txt 2>&1 || exit 3
  echo "== $v"; grep -v amdgpu.ids $OUT/dw_$v.txt | head -12
done
for r in 1 2; do for v in base ns3 ns4; do
  lib=$L/libnerf_hip.so; [ $v = base ] || lib=$L/ab/$v.so
  NERF_HIP_LIB=$lib timeout -k 10 150 python -u scripts/step_ab.py --steps 20 --rounds 3 --settings default > $OUT/step_${v}_$r.txt 2>&1 || exit 4
  echo "$v round $r: $(grep -o '"ms_per_step_median": [0-9.]*' $OUT/step_${v}_$r.txt)"
done; done
