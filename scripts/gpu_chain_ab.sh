set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out
mkdir -p $OUT
for c in 1 0 1; do
  NERF_CHAIN=$c timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-alt > $OUT/ab_$c.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('$OUT/ab_$c.json')); print('chain=$c', round(d['value']), round(d['ms_per_step'],3))"
done
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_chain -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt > $OUT/prof_chain.json 2> $OUT/prof_chain.err && echo "prof ok"
