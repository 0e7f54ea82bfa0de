# round-2 GPU call AE: NT epilogue phase stamps (diagnostic build)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02ae
mkdir -p $OUT
NERF_HIP_LIB=$R/my-nope-nerf_amd/lib/ab/stamps.so timeout -k 10 300 python scripts/nt_bench.py --stamps > $OUT/nt.txt 2>&1; rc=$?; cat $OUT/nt.txt | tail -5; exit $rc
