#!/bin/bash
# round 3: A factors on a side stream under the backward (KFAC(early_factors=True)):
# bitwise test, graph tests, bench with and without, window profile
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
O=gpurun_out/r3
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_factor_determinism.py tests/test_gpu_graphs.py tests/test_gpu_mixed.py tests/test_gpu_kfac.py > $O/tests_early.log 2>&1; rc=$?
tail -2 $O/tests_early.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --early-factors 1 > $O/bench20_early.log 2>&1 || { tail -20 $O/bench20_early.log; exit 1; }
tail -1 $O/bench20_early.log | cut -c1-900
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --early-factors 0 > $O/bench20_noearly.log 2>&1 || { tail -20 $O/bench20_noearly.log; exit 1; }
tail -1 $O/bench20_noearly.log | cut -c1-900
