# One GPU box call, parametrised: scripts/gpu/check.sh TAG STEP [STEP ...]
# STEPs (run in order, each under its own time limit, stopping at the first failure):
#   tests   the full -m gpu suite          smoke  __graft_entry__.smoke()
#   bench   the default bench.py line      prof   rocprofv3 kernel stats of a short eager bench
#   full    scripts/bench_full.py (cfg3)   t:<pytest node or -k expr>  a subset of the GPU tests
#   py:<script args>  python <script args> (under scripts/)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
TAG=$1; shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
n=0
for step in "$@"; do
  case "$step" in
    tests)
      timeout -k 10 800 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.txt 2>&1
      rc=$?; tail -3 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc ;;
    t:*)
      n=$((n + 1))
      timeout -k 10 600 python -u -m pytest ${step#t:} -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tsub$n.txt 2>&1
      rc=$?; tail -3 $OUT/tsub$n.txt; [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
      tail -1 $OUT/smoke.log ;;
    bench)
      timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
      python -c "import json;d=json.load(open('$OUT/bench.json'));print('bench', d['value'], d['ms_per_step'], d.get('ms_per_step_median'), d['execution'], d['roofline']['frac'], d.get('render_cfg4',{}).get('ms_per_frame'), d.get('full_cfg3',{}).get('ms_per_step'))" ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_bench -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt --exec eager > $OUT/prof_bench.log 2>&1) || exit $?
      echo "prof ok" ;;
    full)
      timeout -k 10 300 python -u scripts/bench_full.py --steps 40 --warmup 5 > $OUT/bench_full.json 2> $OUT/bench_full.err || exit $?
      tail -1 $OUT/bench_full.json ;;
    py:*)
      args=${step#py:}
      (cd $R/scripts && timeout -k 10 300 python -u $args > $OUT/py_$(echo $args | tr ' /' '__' | cut -c1-60).txt 2>&1) || exit $?
      echo "py ok: $args" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
