#!/bin/bash
# round 3: grouped SYRK k-step configurations (KFAC_SYRK_CFG 0..3): factor tests
# under each, factor-step time on ResNet-50; then the language models
set -o pipefail
mkdir -p gpurun_out/r3
O=gpurun_out/r3
for cfg in 0 1 2 3; do
  KFAC_SYRK_CFG=$cfg timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_factor_determinism.py tests/test_gpu_kernels.py > $O/tests_syrk$cfg.log 2>&1; rc=$?
  echo "cfg $cfg tests rc=$rc"; tail -1 $O/tests_syrk$cfg.log
  [ $rc -eq 0 ] || exit $rc
  KFAC_SYRK_CFG=$cfg timeout -k 10 200 python -u scripts/probes/probe_factors.py > $O/factors_cfg$cfg.log 2>&1 || { tail -20 $O/factors_cfg$cfg.log; exit 1; }
  grep -v amdgpu.ids $O/factors_cfg$cfg.log
done
