# round-3 GPU call ZC: TN weight-gradient ablations (bias sums; the operand split via a diagnostic build)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03zc
mkdir -p $OUT
for r in 1 2; do
  timeout -k 10 100 python -u scripts/tn_ablation.py 2> /dev/null | tail -1 || exit 3
  NERF_HIP_LIB=$R/my-nope-nerf_amd/lib/ab/tnab.so timeout -k 10 100 python -u scripts/tn_ablation.py 2> /dev/null | tail -1 || exit 3
done
