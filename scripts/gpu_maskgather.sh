set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_render.py -q -x -p no:cacheprovider > gpurun_out/t_mg.log 2>&1; rc=$?
tail -3 gpurun_out/t_mg.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/gemm_bench.py --x6 > gpurun_out/gb_mg.txt 2>&1 && grep "policy 3" gpurun_out/gb_mg.txt && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch -o run -- python $R/scripts/gemm_bench.py --quick --x6 > $R/gpurun_out/pmc_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write -o run -- python $R/scripts/gemm_bench.py --quick --x6 > $R/gpurun_out/pmc_write.log 2>&1 && echo pmc ok
