# round-3 GPU call ZB: the input gradient as eight-wave 128 x 256 tiles (2 or 4 waves per SIMD)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03zb
mkdir -p $OUT
L=$R/my-nope-nerf_amd/lib
for r in 1 2; do for v in base 8w2 8w4; do
  lib=$L/libnerf_hip.so; [ $v = base ] || lib=$L/ab/$v.so
  NERF_HIP_LIB=$lib timeout -k 10 100 python -u scripts/nt_bench.py --iters 30 > $OUT/nt_${v}_$r.json 2> $OUT/nt_${v}_$r.err || exit 3
  echo "$v nt round $r: $(cat $OUT/nt_${v}_$r.json)"
done; done
NERF_HIP_LIB=$L/ab/8w2.so timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x -k "bwd_data" --timeout 100 -p no:cacheprovider 2>&1 | tail -2
