#!/bin/bash
# round 3: channel-major BN chunk partials (finalize reads contiguous runs):
# BN tests, driver bench, window profile
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
O=gpurun_out/r3
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bn.py tests/test_gpu_mixed.py > $O/tests_bn.log 2>&1; rc=$?
tail -2 $O/tests_bn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench20_bn.log 2>&1 || { tail -20 $O/bench20_bn.log; exit 1; }
tail -1 $O/bench20_bn.log
STEPS=20 bash scripts/gpu_prof.sh > $O/prof_bn_summary.log 2>&1; rc=$?; head -16 gpurun_out/prof_bench/window_summary.txt; grep -A5 "batchnorm" gpurun_out/prof_bench/window_summary.txt | tail -5; exit $rc
