# round-3 GPU call S: host enqueue split of the cfg2 step (field forward / backward / rest) and
# the PMC HBM bytes of the GEMM launches incl. the two-segment weight gradients
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03s
mkdir -p $OUT
timeout -k 10 120 python -u scripts/host_split.py > $OUT/host_split.json 2> $OUT/host_split.err; echo host rc=$?; cat $OUT/host_split.json
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex 'k_gemm_(nt|tn)_x6|k_mlp_chain_train2' --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run -- python3 $R/bench.py --steps 3 --warmup 2 --no-alt --no-cpu-baseline --exec eager > $OUT/pmc_fetch.log 2>&1 && echo "pmc fetch ok" && \
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex 'k_gemm_(nt|tn)_x6|k_mlp_chain_train2' --pmc WRITE_SIZE -d $OUT/pmc_write -o run -- python3 $R/bench.py --steps 3 --warmup 2 --no-alt --no-cpu-baseline --exec eager > $OUT/pmc_write.log 2>&1 && echo "pmc write ok"
