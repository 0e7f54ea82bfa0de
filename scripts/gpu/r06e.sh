# round 6: spreading the training chains' vector-memory issue -- the second store of a saved pair
# STSPLIT tiles after the first, the second DMA half DMA2 tiles after the barrier (lib A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06e; mkdir -p $O
(cd scripts && timeout -k 10 1100 python -u lib_ab.py --rounds 2 --steps 20 my-nope-nerf_amd/lib/ab/st1.so my-nope-nerf_amd/lib/ab/st2.so my-nope-nerf_amd/lib/ab/dma2.so my-nope-nerf_amd/lib/ab/st2dma2.so > ../$O/spread_ab.txt 2>&1) || exit $?
grep median $O/spread_ab.txt
