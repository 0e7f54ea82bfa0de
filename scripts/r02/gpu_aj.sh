# round-2 GPU call AJ: backward tail schedule re-tuned after the heads split; kernel trace of the current tree
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02aj
mkdir -p $OUT
timeout -k 10 600 python scripts/step_ab.py --steps 30 --rounds 5 --settings default tail1 tail3 tail2_ts1 tail1_ts2 tside2 > $OUT/sched.json 2> $OUT/sched.err && cat $OUT/sched.json && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt > $OUT/prof_bench.json 2> $OUT/prof.err && echo "prof ok"
