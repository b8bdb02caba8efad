#!/bin/bash
# End-of-session validation: full GPU suite, smoke, driver-command bench, window profile.
# Stops at the first failing step.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=10 > gpurun_out/pytest_gpu_full.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/pytest_gpu_full.log; tail -14 gpurun_out/pytest_gpu_full.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench20.log 2>&1 || { tail -20 gpurun_out/bench20.log; exit 1; }
tail -1 gpurun_out/bench20.log
STEPS=20 bash scripts/gpu_prof.sh > gpurun_out/prof_bench_summary.log 2>&1; rc=$?; tail -30 gpurun_out/prof_bench_summary.log; exit $rc
