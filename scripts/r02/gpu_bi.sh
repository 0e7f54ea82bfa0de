# round-2 GPU call BI: HBM bytes of the fused per-ray eval render (cfg4) from PMC passes (FETCH_SIZE / WRITE_SIZE)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02bi
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
CMD="python3 $R/scripts/bench_render.py --frames 2 --warmup 1"
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run -- $CMD > $OUT/pmc_fetch.log 2>&1 && echo "pmc fetch ok" && \
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d $OUT/pmc_write -o run -- $CMD > $OUT/pmc_write.log 2>&1 && echo "pmc write ok"
