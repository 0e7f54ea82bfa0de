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
    pmc:*)
      # one PMC pass (its own run, --kernel-trace only): pmc:<set> with the sets below
      C1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS"
      C2="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT"
      BENCH="$R/bench.py --steps 3 --warmup 2 --no-alt --no-cpu-baseline --no-cfg3 --exec eager"
      STEPRX='k_gemm_(nt|tn)_x6|k_wgrad|k_mlp_chain'
      case "${step#pmc:}" in
        wg1) RX=k_wgrad_pair; CT="$C1"; CMD="$R/scripts/wgrad_bench.py --loop 20" ;;
        wg2) RX=k_wgrad_pair; CT="$C2"; CMD="$R/scripts/wgrad_bench.py --loop 20" ;;
        wgf) RX=k_wgrad_pair; CT="FETCH_SIZE"; CMD="$R/scripts/wgrad_bench.py --loop 20" ;;
        wgw) RX=k_wgrad_pair; CT="WRITE_SIZE"; CMD="$R/scripts/wgrad_bench.py --loop 20" ;;
        wgh) RX=k_wgrad_pair; CT="TCC_HIT_sum TCC_MISS_sum"; CMD="$R/scripts/wgrad_bench.py --loop 20" ;;
        wj1) RX=k_wgrad_jobs; CT="$C1"; CMD="$BENCH" ;;
        wj2) RX=k_wgrad_jobs; CT="$C2"; CMD="$BENCH" ;;
        wj3) RX=k_wgrad_jobs; CT="SQ_WAVES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES"; CMD="$BENCH" ;;
        lds) RX='k_'; CT="SQ_WAVES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES"; CMD="$BENCH" ;;
        ch1) RX=k_mlp_chain; CT="$C1"; CMD="$BENCH" ;;
        ch2) RX=k_mlp_chain; CT="$C2"; CMD="$BENCH" ;;
        ch3) RX=k_mlp_chain; CT="SQ_WAVES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_VALU_MFMA_COEXEC_CYCLES SQ_BUSY_CYCLES"; CMD="$BENCH" ;;
        ch4) RX=k_mlp_chain; CT="SQ_WAVES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_LDS_ATOMIC SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE"; CMD="$BENCH" ;;
        ic) RX=k_mlp_chain; CT="SQ_WAVES SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAIT_INST_ANY SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE"; CMD="$BENCH" ;;
        fetch) RX="$STEPRX"; CT="FETCH_SIZE"; CMD="$BENCH" ;;
        write) RX="$STEPRX"; CT="WRITE_SIZE"; CMD="$BENCH" ;;
        *) echo "unknown pmc set $step"; exit 2 ;;
      esac
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex "$RX" --pmc $CT -d $OUT/pmc_${step#pmc:} -o run -- python3 $CMD > $OUT/pmc_${step#pmc:}.log 2>&1) || exit $?
      echo "pmc ok: ${step#pmc:}" ;;
    conv:*)
      # the PSNR convergence study (tests/convergence_study.py, 8000 annealed steps): conv:<seeds>
      seeds=$(echo ${step#conv:} | tr ',' ' ')
      timeout -k 10 1100 python -u tests/convergence_study.py --steps 8000 --seeds $seeds --widths 256 --modes f32 f16x3 \
        --window 1000 --every-late 100 --every 100 --lr-milestones 0.4 0.55 0.7 --lr-gamma 0.2 \
        > $OUT/conv_$(echo $seeds | tr ' ' '_').jsonl 2> $OUT/conv_$(echo $seeds | tr ' ' '_').log || exit $?
      tail -1 $OUT/conv_$(echo $seeds | tr ' ' '_').jsonl ;;
    list)
      (cd /tmp && timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1) || exit $?
      echo "list ok" ;;
    py:*)
      args=${step#py:}
      (cd $R/scripts && timeout -k 10 1000 python -u $args > $OUT/py_$(echo $args | tr ' /' '__' | cut -c1-60).txt 2>&1) || exit $?
      echo "py ok: $args" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
