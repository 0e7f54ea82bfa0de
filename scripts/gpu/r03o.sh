# round-3 GPU call O: the two-segment weight gradient in one launch (nerf_linear_bwd_weight_seg):
# kernel tests, the full-step / render gradient tests, an interleaved step A/B against the
# two-launch path, and a kernel trace of the step
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03o
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_full_step.py tests/test_gpu_render.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests.txt 2>&1; rc=$?; tail -3 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/step_ab.py --steps 20 --rounds 5 --settings default dw_two_launch > $OUT/step_ab.txt 2>&1 && tail -4 $OUT/step_ab.txt || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-alt --exec eager > $OUT/trace.log 2>&1 && echo "trace ok" && \
python3 $R/scripts/timeline.py $OUT/trace/run_kernel_trace.csv > $OUT/timeline.txt 2>&1; echo timeline rc=$?
