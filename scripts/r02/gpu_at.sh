# round-2 GPU call AT: sources of the torch glue kernels in cfg3 / cfg2 (torch.profiler stacks)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02at
mkdir -p $OUT
timeout -k 10 300 python scripts/glue_sources.py --full > $OUT/glue_cfg3.txt 2> $OUT/glue_cfg3.err; rc=$?; head -90 $OUT/glue_cfg3.txt; tail -3 $OUT/glue_cfg3.err; exit $rc
