# round-3 GPU call ZA: bench.py with the config-4 render line
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03za
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-alt --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err && python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['ms_per_step'], json.dumps(d['render_cfg4']))"
