# round 6: the weight-gradient groups A/B with one fresh bench process per setting and round
# (same seeds, same data; eager and graph): one list, second launch grouped, both grouped
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06m; mkdir -p $O
(cd scripts && timeout -k 10 1000 python -u lib_ab.py --rounds 3 --steps 30 --exec auto env:NERF_WGRAD_GROUPS=1 env:NERF_WGRAD_GROUPS=2 > ../$O/groups_lib_ab.txt 2>&1) || exit $?
grep median $O/groups_lib_ab.txt
