# round-2 GPU call AS: input-gradient chain on a high-priority stream (NERF_CHAIN_PRIORITY) vs default, same box
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02as
mkdir -p $OUT
for r in 1 2 3 4; do
  for cp in 1 0; do
    NERF_CHAIN_PRIORITY=$cp timeout -k 10 300 python bench.py --no-alt --no-cpu-baseline --exec eager --steps 60 > $OUT/b.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.load(open('$OUT/b.json')); print('chain_prio=$cp', round(d['ms_per_step'],4), {k: round(v['avg_launch_us'],1) for k,v in d['roofline']['per_kind'].items()})" | tee -a $OUT/step_ab.txt
  done
done
