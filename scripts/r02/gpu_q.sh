# round-2 GPU call Q: co-resident block stagger A/B (NT fwd / dX microbench, then the step)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02q
mkdir -p $OUT
for st in 0 8000 16000 24000 40000 64000; do
  NERF_NT_STAGGER=$st NERF_NT_STAGGER_BWD=$st timeout -k 10 120 python -u scripts/nt_bench.py >> $OUT/nt.jsonl 2>> $OUT/nt.err || exit 1
done
cat $OUT/nt.jsonl
for st in 0 16000 32000; do
  NERF_NT_STAGGER=$st NERF_NT_STAGGER_BWD=$st timeout -k 10 200 python -u scripts/step_ab.py --steps 20 --rounds 3 --settings default > $OUT/step_$st.json 2> $OUT/step_$st.err || exit 1
  echo "step stagger=$st $(tail -1 $OUT/step_$st.json)"
done
