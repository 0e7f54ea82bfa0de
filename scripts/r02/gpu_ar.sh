# round-2 GPU call AR: cfg3 kernel trace (graph replay) of the current tree
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02ar
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/scripts/bench_full.py --steps 10 --warmup 3 --mode eager > $OUT/full.json 2> $OUT/full.err && echo "prof ok"
