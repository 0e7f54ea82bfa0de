# round-3 GPU call ZF: the tail (weight gradients of the last layers on the main stream) under the native backward
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03zf
mkdir -p $OUT
timeout -k 10 400 python -u scripts/step_ab.py --steps 20 --rounds 5 --settings default tail1 tail3 > $OUT/step_ab.txt 2>&1 && tail -1 $OUT/step_ab.txt
