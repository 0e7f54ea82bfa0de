# round-2 GPU call AD: NT epilogue cost split (diagnostic builds: 8 no output stores, 16 no maxima, 24 neither)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02ad
mkdir -p $OUT
L=$R/my-nope-nerf_amd/lib
for lib in $L/libnerf_hip.so $L/ab/ablate8.so $L/ab/ablate16.so $L/ab/ablate24.so $L/libnerf_hip.so; do
  echo -n "$(basename $lib) " >> $OUT/nt.txt
  NERF_HIP_LIB=$lib timeout -k 10 300 python scripts/nt_bench.py >> $OUT/nt.txt 2>/dev/null || exit 1
done
NERF_HIP_LIB=$L/libnerf_hip.so timeout -k 10 300 python scripts/nt_bench.py --ablate 1 >> $OUT/nt.txt 2>/dev/null
cat $OUT/nt.txt
