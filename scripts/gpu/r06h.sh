# round 6: the grouped second weight-gradient launch (NERF_WGRAD_GROUPS=1): the slab bit-identity tests,
# the native backward / full-step parity with the groups on, then an eager + graph A/B of the cfg2 step
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06h; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "wgrad_jobs" -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $O/wgrad_tests.txt 2>&1 || exit $?
tail -1 $O/wgrad_tests.txt
NERF_WGRAD_GROUPS=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_native_bwd.py tests/test_gpu_full_step.py tests/test_gpu_render.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/groups_tests.txt 2>&1 || exit $?
tail -1 $O/groups_tests.txt
(cd scripts && timeout -k 10 600 python -u graph_env_ab.py --rounds 3 --steps 30 default NERF_WGRAD_GROUPS=1 > ../$O/groups_ab.json 2> ../$O/groups_ab.err) || exit $?
python -c "import json;d=json.load(open('$O/groups_ab.json'));print({k:{m:round(v['ms_per_step_median'],4) for m,v in r.items()} for k,r in d.items()})"
(cd scripts && timeout -k 10 400 python -u graph_timing_probe.py --rounds 3 --steps 30 > ../$O/graph_timing.json 2> ../$O/graph_timing.err) || exit $?
python -c "import json;d=json.load(open('$O/graph_timing.json'));print({k:{m:round(v['median'],4) for m,v in r.items() if m!='checks'} for k,r in d.items()})"
