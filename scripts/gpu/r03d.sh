# round-3 GPU call D: PSNR convergence at D = 256: 8000 steps x 3 seeds,
# exact f32 and f16x3 against the oracle run by torch on the GPU (+ the chunked-oracle
# control), one MultiStepLR (x0.3 at 50 % and 75 %) on every side so the curves plateau
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03d
mkdir -p $OUT
timeout -k 10 1140 python -u tests/convergence_study.py --widths 256 --seeds 0 1 2 --modes f32 f16x3 --steps 8000 \
  --every 500 --window 1000 --every-late 100 --lr-milestones 0.5 0.75 --lr-gamma 0.3 \
  > $OUT/convergence_8000steps.jsonl 2> $OUT/convergence_8000steps.log
rc=$?; tail -3 $OUT/convergence_8000steps.log; tail -c 1500 $OUT/convergence_8000steps.jsonl; exit $rc
