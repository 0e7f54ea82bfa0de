# round 6: the PSNR parity study on the round-6 tree (block-grouped weight gradients change the
# split sums' order): f16x3 against the fp32 oracle and its 64k-chunk control, seeds from $1
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06v; mkdir -p $O
seeds=$(echo $1 | tr ',' ' ')
tag=$(echo $1 | tr ',' '_')
timeout -k 10 1150 python -u tests/convergence_study.py --steps 8000 --seeds $seeds --widths 256 --modes f16x3 \
  --window 1000 --every-late 100 --every 100 --lr-milestones 0.4 0.55 0.7 --lr-gamma 0.2 \
  > $O/conv_$tag.jsonl 2> $O/conv_$tag.log || exit $?
tail -1 $O/conv_$tag.jsonl
