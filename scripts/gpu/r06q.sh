# round 6: cfg3 host enqueue (plain timing and cProfile) and kernel traces of the cfg3 step eager
# and as graph replays (verdict item 7: where the graph's extra GPU time goes)
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=gpurun_out/r06q; mkdir -p $O
(cd scripts && timeout -k 10 300 python -u host_profile.py --full --plain > ../$O/host_cfg3_plain.txt 2>&1) || exit $?
tail -1 $O/host_cfg3_plain.txt
(cd scripts && timeout -k 10 300 python -u host_profile.py --full --same-thread > ../$O/host_cfg3_prof.txt 2>&1) || exit $?
head -1 $O/host_cfg3_prof.txt
for m in eager graph; do
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/trace_$m -o run -- python3 $R/scripts/bench_full.py --steps 20 --warmup 5 --mode $m > $R/$O/trace_$m.log 2>&1) || exit $?
  echo "trace ok $m"
done
