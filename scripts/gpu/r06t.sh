# round 6: the colour layer's two weight-gradient segments as every-group jobs in launch 1
# (each group half of its 2 S splits; 4.75 / 4.75 tile-times) against f in group 0 and enc_d in
# group 1 (5 / 4.5; lib/ab/old.so) and the l4 .. l0 launch first (NERF_WGRAD_ORDER=1): job-list
# kernel tests, native backward, then the A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06t; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "wgrad or slab or weight" > $O/ktests.txt 2>&1 || exit $?
tail -1 $O/ktests.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_native_bwd.py tests/test_gpu_full_step.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1 || exit $?
tail -1 $O/tests.txt
(cd scripts && timeout -k 10 900 python -u lib_ab.py --rounds 3 --steps 30 my-nope-nerf_amd/lib/ab/old.so env:NERF_WGRAD_ORDER=1 > ../$O/colour_ab.txt 2>&1) || exit $?
grep median $O/colour_ab.txt
