# round 6: launch 2's groups re-assigned so both reads of l4's dy start together (group 0 l4 h3 +
# l3 + l0, group 1 l4 enc_p + l2 + l1; narrow jobs first under groups) against the previous
# assignment (lib/ab/old.so), fresh processes interleaved; native-backward tests first
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06s; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_native_bwd.py tests/test_gpu_full_step.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1 || exit $?
tail -1 $O/tests.txt
(cd scripts && timeout -k 10 900 python -u lib_ab.py --rounds 3 --steps 30 my-nope-nerf_amd/lib/ab/old.so > ../$O/l4_ab.txt 2>&1) || exit $?
grep median $O/l4_ab.txt
