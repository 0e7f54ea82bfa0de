# round 6: both slab-reduce batches in one launch after the second weight-gradient launch (the
# default now) against the first batch between the launches (NERF_WGRAD_BATCH1=1), fresh processes;
# the native-backward tests; then the cfg3 host profile (plain enqueue timing and cProfile)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06p; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_native_bwd.py tests/test_gpu_full_step.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1 || exit $?
tail -1 $O/tests.txt
(cd scripts && timeout -k 10 900 python -u lib_ab.py --rounds 3 --steps 30 env:NERF_WGRAD_BATCH1=1 > ../$O/batch_ab.txt 2>&1) || exit $?
grep median $O/batch_ab.txt
(cd scripts && timeout -k 10 300 python -u host_profile.py --full --plain > ../$O/host_cfg3_plain.txt 2>&1) || exit $?
cat $O/host_cfg3_plain.txt | tail -1
(cd scripts && timeout -k 10 300 python -u host_profile.py --full --same-thread > ../$O/host_cfg3_prof.txt 2>&1) || exit $?
head -3 $O/host_cfg3_prof.txt
