#!/bin/bash
# BN kernel change check: fused-BN / graph / ResNet-50 parity tests, the
# driver-command bench, and the bench-window kernel breakdown.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_bn.py tests/test_gpu_graphs.py tests/test_gpu_resnet50_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/bn_tests.log 2>&1; rc=$?; tail -3 gpurun_out/bn_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench20_bn.log 2>&1 && tail -1 gpurun_out/bench20_bn.log &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench20_bn_rep.log 2>&1 && tail -1 gpurun_out/bench20_bn_rep.log &&
STEPS=20 bash scripts/gpu_prof.sh > gpurun_out/prof_bn_summary.log 2>&1; grep -A6 "batchnorm" gpurun_out/prof_bn_summary.log | head -12
