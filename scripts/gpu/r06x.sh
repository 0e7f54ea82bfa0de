# round 6: the first weight-gradient launch's load waves four stages ahead (NS 4 in
# k_wgrad_jobs<3>, no spill; <6> spills at 4 and keeps 3): job-list kernel tests through that
# library, then the A/B against the tree's library
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=gpurun_out/r06x; mkdir -p $O
NERF_HIP_LIB=$R/my-nope-nerf_amd/lib/ab/ns4j.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_native_bwd.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "wgrad or weight or native" > $O/ns4j_tests.txt 2>&1 || exit $?
tail -1 $O/ns4j_tests.txt
(cd scripts && timeout -k 10 900 python -u lib_ab.py --rounds 3 --steps 30 my-nope-nerf_amd/lib/ab/ns4j.so > ../$O/ns4j_ab.txt 2>&1) || exit $?
grep median $O/ns4j_ab.txt
