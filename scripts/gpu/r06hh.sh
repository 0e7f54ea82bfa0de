# round 6: the fused eval kernel's encoding tile with swizzled float4 chunks (the prologue's
# per-row writes off one bank): chain / render tests through the variant, its LDS counters, then
# the A/B (the render frame is in each line)
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=gpurun_out/r06hh; mkdir -p $O
NERF_HIP_LIB=$R/my-nope-nerf_amd/lib/ab/encswz.so timeout -k 10 500 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_render.py tests/test_gpu_distributed.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -k "not process_group_matches" > $O/encswz_tests.txt 2>&1 || exit $?
tail -1 $O/encswz_tests.txt
(cd scripts && timeout -k 10 900 python -u lib_ab.py --rounds 3 --steps 20 my-nope-nerf_amd/lib/ab/encswz.so > ../$O/encswz_ab.txt 2>&1) || exit $?
grep median $O/encswz_ab.txt
grep frame $O/encswz_ab.txt | awk '{print $2, $6}'
