#!/bin/bash
# End-of-session check on the final tree: full GPU suite, smoke, the driver
# bench command, and a 2-rank gloo rehearsal of the multi-rank bench path.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_end.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu_end.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_end.log 2>&1 && tail -1 gpurun_out/smoke_end.log &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench20_end.log 2>&1 && tail -1 gpurun_out/bench20_end.log | cut -c1-300 &&
N=2 bash scripts/gpu_rehearse_multirank.sh
