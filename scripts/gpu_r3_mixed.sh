#!/bin/bash
# round 3: bf16-stored weights with fp32 masters (ops/mixed.py): GPU tests, bench on / off
set -o pipefail
mkdir -p gpurun_out/r3
O=gpurun_out/r3
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_mixed.py tests/test_gpu_graphs.py tests/test_gpu_overlap_precond.py > $O/tests_mixed.log 2>&1; rc=$?
tail -3 $O/tests_mixed.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench20_bf16w.log 2>&1 || { tail -20 $O/bench20_bf16w.log; exit 1; }
tail -1 $O/bench20_bf16w.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --bf16-weights 0 > $O/bench20_autocast.log 2>&1 || { tail -20 $O/bench20_autocast.log; exit 1; }
tail -1 $O/bench20_autocast.log
N=2 bash scripts/gpu_rehearse_multirank.sh &&
N=4 BENCH_ARGS="--comm-method hybrid-opt --grad-worker-fraction 0.5" bash scripts/gpu_rehearse_multirank.sh
