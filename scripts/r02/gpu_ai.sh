# round-2 GPU call AI: dyr gated by the colour layer's ReLU bits -- parity, then the same-box A/B of the schedule
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02ai
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_full_step.py tests/test_gpu_render.py tests/test_gpu_graph.py > $OUT/tests.txt 2>&1; rc=$?; tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3 4; do
  for hs in 1 0; do
    NERF_HEADS_SIDE=$hs timeout -k 10 300 python bench.py --no-alt --no-cpu-baseline --steps 60 > $OUT/b.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.load(open('$OUT/b.json')); print('heads_side=$hs', round(d['ms_per_step'],4), {k: round(v['avg_launch_us'],1) for k,v in d['roofline']['per_kind'].items()})" | tee -a $OUT/step_ab.txt
  done
done
