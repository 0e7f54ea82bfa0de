# round 6: head-weight partial placements on the final weight-gradient schedule (the slab
# reduces now one launch at the end): 5 (default) vs 3 (k_heads_part, 16-byte loads, reduces
# with the slabs) vs 1 (partials + reduce before the chain), fresh processes interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06y; mkdir -p $O
(cd scripts && timeout -k 10 1000 python -u lib_ab.py --rounds 3 --steps 30 env:NERF_HEADS_PLACE=3 env:NERF_HEADS_PLACE=1 > ../$O/heads_ab.txt 2>&1) || exit $?
grep median $O/heads_ab.txt
