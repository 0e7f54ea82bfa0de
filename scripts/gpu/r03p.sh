# round-3 GPU call P: every layer's slab reduce in one launch at the end of the backward
# (nerf_slab_reduce_batch) + the two-segment weight gradient: kernel / full-step / render /
# distributed tests, an interleaved step A/B over the schedule switches, a kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03p
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_full_step.py tests/test_gpu_render.py tests/test_gpu_distributed.py tests/test_gpu_graph.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests.txt 2>&1; rc=$?; tail -3 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/step_ab.py --steps 20 --rounds 5 --settings default slab_per_layer batch_tail1 batch_tail0 > $OUT/step_ab.txt 2>&1 && tail -2 $OUT/step_ab.txt || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-alt --exec eager > $OUT/trace.log 2>&1 && echo "trace ok" && \
python3 $R/scripts/timeline.py $OUT/trace/run_kernel_trace.csv > $OUT/timeline.txt 2>&1; echo timeline rc=$?
