# round 6: k_pack's grid (f32-copy blocks x image blocks per descriptor: 128 x 128 in the tree)
# against 64 x 128, 128 x 256 and 32 x 64, fresh processes interleaved; the pack tests through
# each variant first
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=gpurun_out/r06z; mkdir -p $O
for v in pk64_128 pk128_256 pk32_64; do
  NERF_HIP_LIB=$R/my-nope-nerf_amd/lib/ab/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_chain.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "pack or chain_matches" > $O/tests_$v.txt 2>&1 || exit $?
  tail -1 $O/tests_$v.txt
done
(cd scripts && timeout -k 10 1000 python -u lib_ab.py --rounds 3 --steps 30 my-nope-nerf_amd/lib/ab/pk64_128.so my-nope-nerf_amd/lib/ab/pk128_256.so my-nope-nerf_amd/lib/ab/pk32_64.so > ../$O/pack_ab.txt 2>&1) || exit $?
grep median $O/pack_ab.txt
