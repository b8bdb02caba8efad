#!/bin/bash
# One GPU-box session: GPU tests, smoke, headline bench (K-FAC and SGD-only),
# rocprofv3 kernel breakdown of the timed window, eigensolver backend probe.
# Every GPU step has its own time limit; the first failure ends the session.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "$name failed rc=$rc"; exit $rc; fi
}
STEPS=${STEPS:-100}
if [ -z "$SKIP_TESTS" ]; then
  run pytest_gpu 540 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
  run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ -z "$SKIP_BENCH" ]; then
  run bench_kfac 300 python bench.py --steps $STEPS --warmup 10 $BENCH_ARGS
  run bench_sgd 200 python bench.py --steps $STEPS --warmup 10 --no-kfac
fi
if [ -n "$PROFILE" ]; then
  rm -rf /tmp/prof_bench
  export KFAC_PROFILE_MARKER=1
  run prof_bench 400 rocprofv3 --kernel-trace -d /tmp/prof_bench -o run --output-format csv -- python3 bench.py --steps $STEPS --warmup 10 $BENCH_ARGS
  unset KFAC_PROFILE_MARKER
  f=$(find /tmp/prof_bench -name "*kernel_trace.csv" | head -1)
  python3 scripts/prof_window.py "$f" $STEPS > gpurun_out/prof_window_summary.txt
  head -20 gpurun_out/prof_window_summary.txt
fi
if [ -n "$PROBE_EIGH" ]; then
  run probe_eigh 400 python scripts/probes/probe_eigh_backends.py
fi
echo "session ok"
