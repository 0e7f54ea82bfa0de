# round-2 GPU call AL: cfg3 (full step) under the backward schedule knobs, same box, 3 rounds (graph replay:
# the host is out of the timed loop, eager cfg3 runs at the host's pace on a noisy CPU share)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02al
mkdir -p $OUT
for r in 1 2 3; do
  for cfg in "1 3" "0 3" "1 2" "0 2"; do
    set -- $cfg
    NERF_HEADS_SIDE=$1 NERF_TAIL_MAIN=$2 timeout -k 10 300 python scripts/bench_full.py --steps 40 --warmup 5 --mode graph > $OUT/f.json 2>/dev/null || exit 1
    python -c "import json; f=json.load(open('$OUT/f.json')); r=f['runs']['graph']; print('heads_side=$1 tail=$2', round(r['ms_per_step'],4))" | tee -a $OUT/cfg3_ab.txt
  done
done
