# round-3 GPU call T: the native field backward (nerf_field_backward): bit-identity against the
# Python schedule, the full-step / distributed / graph tests through it, the host split, and an
# interleaved step A/B native vs Python
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03t
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_native_bwd.py tests/test_gpu_full_step.py tests/test_gpu_distributed.py tests/test_gpu_graph.py tests/test_gpu_render.py tests/test_gpu_field_grads.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests.txt 2>&1; rc=$?; tail -15 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/host_split.py > $OUT/host_split.json 2> $OUT/host_split.err; cat $OUT/host_split.json
timeout -k 10 300 python -u scripts/step_ab.py --steps 20 --rounds 5 --settings default python_bwd > $OUT/step_ab.txt 2>&1 && tail -1 $OUT/step_ab.txt || exit 3
