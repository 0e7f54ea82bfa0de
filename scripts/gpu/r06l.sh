# round 6: both weight-gradient launches as two block groups (NERF_WGRAD_GROUPS=2): the native
# backward / full-step / render parity with the groups on, then an eager + graph A/B of the cfg2
# step against the second launch grouped (1), one list (default) and a repeat of the default
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06l; mkdir -p $O
NERF_WGRAD_GROUPS=2 timeout -k 10 500 python -u -m pytest tests/test_gpu_native_bwd.py tests/test_gpu_full_step.py tests/test_gpu_render.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/groups2_tests.txt 2>&1 || exit $?
tail -1 $O/groups2_tests.txt
(cd scripts && timeout -k 10 700 python -u graph_env_ab.py --rounds 3 --steps 30 default NERF_WGRAD_GROUPS=1 NERF_WGRAD_GROUPS=2 default#2 > ../$O/groups_ab.json 2> ../$O/groups_ab.err) || exit $?
python -c "import json;d=json.load(open('$O/groups_ab.json'));print({k:{m:round(v['ms_per_step_median'],4) for m,v in r.items()} for k,r in d.items()})"
