# round-2 GPU call L: TN register pipeline depth (NERF_TN_NS) -- dW microbench, dW parity tests, step A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r02l
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py -k "weight" > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for ns in 1 3; do
  NERF_TN_NS=$ns timeout -k 10 200 python -u scripts/dw_bench.py --h16 > $OUT/dw_ns$ns.txt 2>&1 || exit 1
  echo "ns=$ns"; grep default $OUT/dw_ns$ns.txt
done
NERF_TN_NS=1 timeout -k 10 200 python -u scripts/step_ab.py --steps 20 --rounds 3 --settings default > $OUT/step_ns1.json 2>&1 && cat $OUT/step_ns1.json | tail -1 && \
NERF_TN_NS=3 timeout -k 10 200 python -u scripts/step_ab.py --steps 20 --rounds 3 --settings default > $OUT/step_ns3.json 2>&1 && cat $OUT/step_ns3.json | tail -1
