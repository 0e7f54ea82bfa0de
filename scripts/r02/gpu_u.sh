# round-2 GPU call U: host (enqueue) profile of the cfg3 eager step
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02u
mkdir -p $OUT
timeout -k 10 300 python -u scripts/host_profile.py --full > $OUT/host_full.txt 2> $OUT/host_full.err; rc=$?
head -5 $OUT/host_full.txt; exit $rc
