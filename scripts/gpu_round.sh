#!/bin/bash
# One GPU-box session: tests, smoke, bench (K-FAC and SGD-only), phase breakdown.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --steps 100 --warmup 10 > gpurun_out/bench_kfac.log 2>&1 || { echo bench failed; tail -30 gpurun_out/bench_kfac.log; exit 1; }
tail -1 gpurun_out/bench_kfac.log
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-kfac > gpurun_out/bench_sgd.log 2>&1 || exit 1
tail -1 gpurun_out/bench_sgd.log
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --profile-phases > gpurun_out/bench_phases.log 2>&1 || exit 1
tail -1 gpurun_out/bench_phases.log
