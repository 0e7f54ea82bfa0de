# round-2 GPU call AN: bench.py with eager + graph-replay timing (default auto), twice
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02an
mkdir -p $OUT
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err && echo "bench ok" && \
timeout -k 10 600 python bench.py --no-alt --no-cpu-baseline > $OUT/bench2.json 2> $OUT/bench2.err && echo "bench2 ok" && \
timeout -k 10 300 python scripts/host_profile.py --plain > $OUT/host_cfg2.txt 2>&1 && tail -1 $OUT/host_cfg2.txt
