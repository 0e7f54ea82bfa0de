# round-3 GPU call J: phase stamps of k_render_fused2 and k_mlp_chain_train2 (+ the training
# ablation builds), HBM bytes per launch of the GEMMs and the training chain in the cfg2 step
# (separate FETCH_SIZE / WRITE_SIZE passes)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03j
mkdir -p $OUT
timeout -k 10 200 python -u scripts/chain_bench.py --fused > $OUT/fused2_stamps.txt 2>&1 && cat $OUT/fused2_stamps.txt || exit 3
for lib in libnerf_hip ab/cmrow ab/tr1 ab/tr2 ab/tr3; do
  NERF_HIP_LIB=$R/my-nope-nerf_amd/lib/$lib.so timeout -k 10 120 python -u scripts/chain_bench.py > $OUT/chain_$(basename $lib).txt 2>&1 || exit 3
  echo "$lib"; grep "keep=True" $OUT/chain_$(basename $lib).txt
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex 'k_gemm_(nt|tn)_x6|k_mlp_chain_train2' --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run -- python3 $R/bench.py --steps 3 --warmup 2 --no-alt --no-cpu-baseline --exec eager > $OUT/pmc_fetch.log 2>&1 && echo "pmc fetch ok" && \
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex 'k_gemm_(nt|tn)_x6|k_mlp_chain_train2' --pmc WRITE_SIZE -d $OUT/pmc_write -o run -- python3 $R/bench.py --steps 3 --warmup 2 --no-alt --no-cpu-baseline --exec eager > $OUT/pmc_write.log 2>&1 && echo "pmc write ok"
