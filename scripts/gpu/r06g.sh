# round 6: the new default (compact exponent arrays in the chain images, input-gradient chain column
# maxima over 4 lanes into 4 LDS copies, eval prologue loads ahead of its DMAs): GPU suite, then the
# forward chain's column maxima the same way (lib A/B) and the head-reduce placement eager + graph
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06g; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1 || exit $?
tail -1 $O/tests.txt
(cd scripts && timeout -k 10 1000 python -u lib_ab.py --rounds 2 --steps 20 my-nope-nerf_amd/lib/ab/fcmq4.so my-nope-nerf_amd/lib/ab/mskw9.so my-nope-nerf_amd/lib/ab/fcmq4mskw9.so > ../$O/fcmq_ab.txt 2>&1) || exit $?
grep median $O/fcmq_ab.txt
(cd scripts && timeout -k 10 600 python -u graph_env_ab.py --rounds 3 --steps 30 default NERF_HEADS_PLACE=1 > ../$O/heads_graph_ab.json 2> ../$O/heads_graph_ab.err) || exit $?
grep -A3 '"graph"' $O/heads_graph_ab.json | grep median
