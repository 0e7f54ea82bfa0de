# round 6: rehearsal of bench.py's N-rank path (the driver's scaling runs) on the one-GPU box:
# two ranks under torch.distributed.run, both on cuda:0 with gloo collectives
# (NERF_BENCH_SHARED_GPU=1): the in-place bucket all-reduce through the real HIP backward,
# barriers, max-over-ranks timing and the rank-0 line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06bb; mkdir -p $O
NERF_BENCH_SHARED_GPU=1 timeout -k 10 400 python -u bench.py --gpus 2 --steps 5 --warmup 2 --no-alt --no-cpu-baseline --no-cfg3 > $O/bench2.json 2> $O/bench2.err || exit $?
python -c "import json;d=json.loads([l for l in open('$O/bench2.json') if l.startswith('{')][-1]);print({k:d.get(k) for k in ['n_gpus','world_size','value','ms_per_step','allreduce_ms_per_step','rehearsal']})"
