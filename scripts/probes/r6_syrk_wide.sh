#!/bin/bash
# Round 6: 256-wide grouped SYRK tiles -- factor kernel tests, then the
# ResNet-50 factor step per KFAC_SYRK_WIDE_MIN (0 = all 128-wide).
set -e -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_factor_determinism.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6_syrk_tests.log 2>&1
for W in 0 512 256 1024; do
  KFAC_SYRK_WIDE_MIN=$W PROBE_SPLITS=2048,4096 timeout -k 10 120 python -u scripts/probes/probe_factors.py > gpurun_out/r6_syrk_wide$W.log 2>&1
done
