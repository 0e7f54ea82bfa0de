# round-3 GPU call ZG: per-phase cycles of the TN main loop (diagnostic stamps build)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03zg
mkdir -p $OUT
NERF_HIP_LIB=$R/my-nope-nerf_amd/lib/ab/tst.so timeout -k 10 100 python -u scripts/tn_stamps.py > $OUT/tn_stamps.json 2> $OUT/tn_stamps.err; echo rc=$?; cat $OUT/tn_stamps.json; tail -3 $OUT/tn_stamps.err
timeout -k 10 100 python -u scripts/tn_ablation.py 2>/dev/null | tail -1
NERF_HIP_LIB=$R/my-nope-nerf_amd/lib/ab/tst.so timeout -k 10 100 python -u scripts/tn_ablation.py 2>/dev/null | tail -1
