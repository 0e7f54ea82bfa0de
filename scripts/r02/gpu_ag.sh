# round-2 GPU call AG: forward layer chain, one stream vs rows split over two streams
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02ag
mkdir -p $OUT
timeout -k 10 300 python scripts/dual_stream_bench.py --layers 4 > $OUT/dual.txt 2>&1 && \
timeout -k 10 300 python scripts/dual_stream_bench.py --layers 8 >> $OUT/dual.txt 2>&1; rc=$?; grep -v amdgpu.ids $OUT/dual.txt; exit $rc
