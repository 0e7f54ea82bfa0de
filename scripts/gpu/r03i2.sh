# round-3 GPU call I2 (seeds 3-5 of call I): PSNR convergence at D = 256 on the default path (the
# training chain): 8000 steps x 3 seeds, exact f32 and f16x3 against the oracle run by torch on
# the GPU (+ the chunked-oracle control); the learning rate annealed on every side alike
# (x0.2 at 40 %, 55 % and 70 %) so the last two 1000-step windows sit on the final rate
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03i
mkdir -p $OUT
timeout -k 10 1150 python -u tests/convergence_study.py --widths 256 --seeds 3 4 5 --modes f32 f16x3 --steps 8000 \
  --every 500 --window 1000 --every-late 100 --lr-milestones 0.4 0.55 0.7 --lr-gamma 0.2 \
  > $OUT/convergence_8000steps_annealed_s345.jsonl 2> $OUT/convergence_8000steps_annealed_s345.log
rc=$?; tail -3 $OUT/convergence_8000steps_annealed_s345.log; tail -c 1500 $OUT/convergence_8000steps_annealed_s345.jsonl; exit $rc
