#!/bin/bash
# End-of-session validation: full GPU suite, smoke, driver-command bench,
# eigensolver group probe, window profile.  Stops at the first failing step.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=10 > gpurun_out/pytest_gpu_full.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/pytest_gpu_full.log; tail -14 gpurun_out/pytest_gpu_full.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log || exit 1
bash scripts/gpu_bench_prof.sh
