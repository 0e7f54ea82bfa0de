# round 6: does the head-reduce placement change any result (bit-identical losses, eager and graph,
# placements 5 and 1, same seeds)?  Then the forward chains' epilogue row maxima by v_max3
# (max3.so: chain tests through that library, then the lib A/B against the default)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06i; mkdir -p $O
(cd scripts && timeout -k 10 400 python -u determinism_probe.py --steps 150 > ../$O/determinism.json 2> ../$O/determinism.err) || exit $?
head -2 $O/determinism.json
NERF_HIP_LIB=$PWD/my-nope-nerf_amd/lib/ab/max3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_render.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/max3_tests.txt 2>&1 || exit $?
tail -1 $O/max3_tests.txt
(cd scripts && timeout -k 10 600 python -u lib_ab.py --rounds 2 --steps 20 my-nope-nerf_amd/lib/ab/max3.so > ../$O/max3_ab.txt 2>&1) || exit $?
grep median $O/max3_ab.txt
