# round-2 GPU call AF: DPP column-max butterfly -- kernel parity, standalone and in-step A/B vs the previous commit
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02af
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_full_step.py > $OUT/tests.txt 2>&1; rc=$?; tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
BASE=$R/my-nope-nerf_amd/lib/ab/base.so
NEW=$R/my-nope-nerf_amd/lib/libnerf_hip.so
for lib in $BASE $NEW $BASE $NEW; do
  echo -n "$(basename $lib) " >> $OUT/nt.txt
  NERF_HIP_LIB=$lib timeout -k 10 300 python scripts/nt_bench.py >> $OUT/nt.txt 2>/dev/null || exit 1
done
cat $OUT/nt.txt
for r in 1 2 3 4; do
  for lib in $NEW $BASE; do
    NERF_HIP_LIB=$lib timeout -k 10 300 python bench.py --no-alt --no-cpu-baseline --steps 60 > $OUT/b.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.load(open('$OUT/b.json')); print('$(basename $lib)', round(d['ms_per_step'],4), {k: round(v['avg_launch_us'],1) for k,v in d['roofline']['per_kind'].items()})" | tee -a $OUT/step_ab.txt
  done
done
