# round-2 GPU call AB2: base vs working-tree library, cfg2 step only, 5 alternating rounds
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02ab2
mkdir -p $OUT
BASE=$R/my-nope-nerf_amd/lib/ab/base.so
NEW=$R/my-nope-nerf_amd/lib/libnerf_hip.so
for r in 1 2 3 4 5; do
  for lib in $NEW $BASE; do
    NERF_HIP_LIB=$lib timeout -k 10 300 python bench.py --no-alt --no-cpu-baseline --steps 60 > $OUT/b.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.load(open('$OUT/b.json')); print('$(basename $lib)', round(d['ms_per_step'],4), {k: round(v['avg_launch_us'],1) for k,v in d['roofline']['per_kind'].items()})" | tee -a $OUT/step_ab.txt
  done
done
