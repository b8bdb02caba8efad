#!/bin/bash
# round 3 (record): LDS-DMA SYRK variants (KFAC_SYRK_DMA=2/3, since removed) vs the
# register-staged default: factor numerics tests and factor-step time
set -o pipefail
mkdir -p gpurun_out/r3
O=gpurun_out/r3
for v in 0 2 3; do
  KFAC_SYRK_DMA=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_factor_determinism.py tests/test_gpu_resnet50_parity.py > $O/tests_syrkdma$v.log 2>&1; rc=$?
  echo "dma $v tests rc=$rc"; tail -2 $O/tests_syrkdma$v.log
  [ $rc -eq 0 ] || exit $rc
  KFAC_SYRK_DMA=$v timeout -k 10 200 python -u scripts/probes/probe_factors.py > $O/factors_dma$v.log 2>&1 || { tail -20 $O/factors_dma$v.log; exit 1; }
  grep -v amdgpu.ids $O/factors_dma$v.log
done
