# round-3 GPU call Q: where the graph replay of the cfg2 step loses against the eager GPU
# timeline (kernel trace of --exec graph), and the host enqueue time of the eager step
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r03q
mkdir -p $OUT
timeout -k 10 200 python -u scripts/host_profile.py > $OUT/host_profile.txt 2>&1; echo host rc=$?; grep -i "enqueue" $OUT/host_profile.txt | head -3
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_graph -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-alt --exec graph > $OUT/trace_graph.log 2>&1 && echo "trace ok" && tail -c 400 $OUT/trace_graph.log
