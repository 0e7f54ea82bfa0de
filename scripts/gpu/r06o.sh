# round 6: the slab reduce with four split loads in flight (the grouped weight gradients' 64-split
# slabs) against the round's previous reduce (lib/ab/slab_old.so), fresh processes, interleaved;
# then the slab / weight-gradient kernel tests
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06o; mkdir -p $O
(cd scripts && timeout -k 10 900 python -u lib_ab.py --rounds 3 --steps 30 my-nope-nerf_amd/lib/ab/slab_old.so > ../$O/slab_ab.txt 2>&1) || exit $?
grep median $O/slab_ab.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "slab or wgrad or weight" > $O/slab_tests.txt 2>&1 || exit $?
tail -1 $O/slab_tests.txt
