# round 6: the per-half barrier tile (lag) in the training chains -- correctness of the lag builds, then
# interleaved whole-library A/Bs on the cfg2 step
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06d; mkdir -p $O
L=$GRAFT_REPO_ROOT/my-nope-nerf_amd/lib/ab
NERF_HIP_LIB=$L/both8.so timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_native_bwd.py tests/test_gpu_full_step.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $O/both8_tests.txt 2>&1 || exit $?
tail -1 $O/both8_tests.txt
(cd scripts && timeout -k 10 1000 python -u lib_ab.py --rounds 2 --steps 20 my-nope-nerf_amd/lib/ab/trlag8.so my-nope-nerf_amd/lib/ab/trlag4.so my-nope-nerf_amd/lib/ab/bwlag8.so my-nope-nerf_amd/lib/ab/both8.so > ../$O/lag_ab.txt 2>&1) || exit $?
grep median $O/lag_ab.txt
# verdict item 8: k_mlp_chain_bwd's in-step durations with k_heads_reduce forked beside it (5) and on the
# caller's stream before it (1), from kernel traces of the eager cfg2 bench
for hp in 5 1; do
  (cd /tmp && export TMPDIR=/tmp && NERF_HEADS_PLACE=$hp timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/trace_hp$hp -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-alt --no-cfg3 --exec eager > $GRAFT_REPO_ROOT/$O/trace_hp$hp.log 2>&1) || exit $?
done
python scripts/heads_ab.py place5=$(ls $O/trace_hp5/*kernel_trace.csv) place1=$(ls $O/trace_hp1/*kernel_trace.csv) > $O/heads_ab.json && python scripts/timeline.py $(ls $O/trace_hp5/*kernel_trace.csv) --gaps 3 > $O/timeline_hp5.txt
head -3 $O/timeline_hp5.txt
