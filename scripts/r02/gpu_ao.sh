# round-2 GPU call AO: cfg2 host enqueue profile with the backward on the calling thread
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02ao
mkdir -p $OUT
timeout -k 10 300 python scripts/host_profile.py --same-thread > $OUT/host_cfg2.txt 2>&1 && head -3 $OUT/host_cfg2.txt
