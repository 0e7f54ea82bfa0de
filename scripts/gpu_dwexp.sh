cd $GRAFT_REPO_ROOT
for b in 256 128 64; do
  NERF_DW_BLOCKS=$b timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-alt > gpurun_out/dwexp_$b.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/dwexp_$b.json')); print($b, round(d['value']), round(d['ms_per_step'],3))"
done
