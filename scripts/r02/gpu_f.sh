# round-2 GPU call F: dW tiling A/B on the training step, dW microbench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02f
mkdir -p $OUT
timeout -k 10 300 python -u scripts/step_ab.py --steps 20 --rounds 3 > $OUT/step_ab.json 2> $OUT/step_ab.err && echo "ab ok" && cat $OUT/step_ab.json
