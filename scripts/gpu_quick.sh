#!/bin/bash
# quick loop: selected GPU tests + phase-profiled bench
set -o pipefail
mkdir -p gpurun_out
python csrc/build.py || exit 1
timeout -k 10 300 python -m pytest tests -m gpu -x -q ${KTEST:+-k "$KTEST"} > gpurun_out/pytest_quick.log 2>&1 || { tail -40 gpurun_out/pytest_quick.log; exit 1; }
tail -2 gpurun_out/pytest_quick.log
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --profile-phases ${BENCH_ARGS} > gpurun_out/bench_quick.log 2>&1 || { tail -30 gpurun_out/bench_quick.log; exit 1; }
tail -1 gpurun_out/bench_quick.log
