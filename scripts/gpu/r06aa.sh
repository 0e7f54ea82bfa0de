# round 6: the backward's persistent seed (no per-step fill launch) against loss.backward()
# (NERF_SEED_ONE=0), fresh processes interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06aa; mkdir -p $O
(cd scripts && timeout -k 10 900 python -u lib_ab.py --rounds 3 --steps 30 env:NERF_SEED_ONE=0 > ../$O/seed_ab.txt 2>&1) || exit $?
grep median $O/seed_ab.txt
