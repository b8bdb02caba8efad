#!/bin/bash
# One parameterised GPU-box runner (replaces the per-session gpu_*.sh scripts;
# git history keeps them).  Runs the named steps in order, each under its own
# time limit; stops at the first failing step (no GPU step after a fault, an
# abort or a time-out).  Output goes to gpurun_out/<step>.log.
#
#   bash scripts/gpu_run.sh tests smoke bench            # the round-end check
#   bash scripts/gpu_run.sh prof                         # rocprofv3 window breakdown
#   TESTS="tests/test_gpu_eig_dc.py" bash scripts/gpu_run.sh tests
#   BENCH_ARGS="--kfac-update-freq 10" STEPS=50 bash scripts/gpu_run.sh bench
#   PROBE="scripts/probes/probe_two_stage.py --sizes 4608" bash scripts/gpu_run.sh probe probe-prof
#   PMC="SQ_WAVES SQ_BUSY_CYCLES" PMC_CMD="python3 scripts/probes/probe_pgemm.py bf16x3" \
#       bash scripts/gpu_run.sh pmc
#
# Steps: tests smoke bench bench-sgd phases prof probe probe-prof pmc rehearse serialized
#   serialized = race-detection leg: the GPU kernel / K-FAC /
#   eigensolver / graph tests with every kernel launch and copy serialised by
#   the HIP runtime -- a test that passes normally but fails here (or the
#   reverse) points at a missing stream / event dependency.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=${STEPS:-20}
WARMUP=${WARMUP:-5}
TESTS=${TESTS:-tests}

step() {  # step <name> <limit_s> <command...>
  local name=$1 lim=$2; shift 2
  echo "[gpu_run] $name (limit ${lim}s)"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -3 "gpurun_out/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "[gpu_run] $name failed rc=$rc"; exit $rc; fi
}

for s in "$@"; do
  case $s in
    tests) step tests 900 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread ;;
    # the round-end driver's exact command (no timeout plugin flags, fresh MIOpen db)
    driver) MIOPEN_USER_DB_PATH=/tmp/mdb_fresh_$$ step driver 900 python3 -m pytest tests/ -x -q -m gpu -p no:cacheprovider ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py --steps $STEPS --warmup $WARMUP $BENCH_ARGS ;;
    bench-sgd) step bench_sgd 600 python bench.py --steps $STEPS --warmup $WARMUP --no-kfac $BENCH_ARGS ;;
    phases) step phases 600 python bench.py --steps $STEPS --warmup $WARMUP --profile-phases $BENCH_ARGS ;;
    prof)
      rm -rf /tmp/prof_bench
      KFAC_PROFILE_MARKER=1 step prof 900 rocprofv3 --kernel-trace -d /tmp/prof_bench -o run \
        --output-format csv -- python3 bench.py --steps $STEPS --warmup $WARMUP $BENCH_ARGS
      f=$(find /tmp/prof_bench -name "*kernel_trace.csv" | head -1)
      python3 scripts/prof_window.py "$f" $STEPS > gpurun_out/prof_window_summary.txt
      python3 scripts/probes/trace_inverse_start.py "$f" > gpurun_out/prof_inverse_start.txt || true
      head -40 gpurun_out/prof_window_summary.txt ;;
    probe) step probe 600 python -u $PROBE ;;
    probe-prof)
      rm -rf /tmp/prof_probe
      step probe_prof 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_probe -o run \
        --output-format csv -- python3 -u $PROBE
      mkdir -p gpurun_out/prof_probe
      find /tmp/prof_probe -name "*stats*.csv" -exec cp {} gpurun_out/prof_probe/ \;
      head -25 gpurun_out/prof_probe/*kernel_stats.csv | cut -c1-200 ;;
    pmc)
      # PMC="<counters>" PMC_CMD="<program>" [PMC_FILTER=<kernel regex>] [PMC_NAME=<name>]
      name=${PMC_NAME:-pmc}
      filt=()
      [ -n "$PMC_FILTER" ] && filt=(--kernel-include-regex "$PMC_FILTER")
      rm -rf /tmp/pmc_$name
      timeout -s KILL 150 rocprofv3 --pmc $PMC "${filt[@]}" -d /tmp/pmc_$name -o run \
        --output-format csv -- $PMC_CMD > gpurun_out/$name.log 2>&1 || {
          echo "[gpu_run] pmc failed"; tail -5 gpurun_out/$name.log; exit 1; }
      python3 scripts/pmc_summary.py /tmp/pmc_$name gpurun_out/${name}_summary.csv
      cat gpurun_out/${name}_summary.csv | cut -c1-200 ;;
    rehearse) N=${N:-2} step rehearse 600 bash scripts/gpu_rehearse_multirank.sh ;;
    serialized)
      AMD_SERIALIZE_KERNEL=3 AMD_SERIALIZE_COPY=3 step serialized 900 python -u -m pytest -x -q \
        --timeout 240 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
        tests/test_gpu_kfac.py tests/test_gpu_eig_dc.py tests/test_gpu_graphs.py ;;
    *) echo "[gpu_run] unknown step $s"; exit 2 ;;
  esac
done
