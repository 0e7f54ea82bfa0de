set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for t in 256 128 64 512; do
  NERF_DW_BLOCKS=$t timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-alt --no-cpu-baseline > gpurun_out/dw_$t.json 2>gpurun_out/dw_$t.err || exit 1
  echo "target $t: $(python -c "import json;d=json.load(open('gpurun_out/dw_$t.json'));print(round(d['value']), round(d['ms_per_step'],3))")"
done
