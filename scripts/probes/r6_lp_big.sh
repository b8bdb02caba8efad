#!/bin/bash
# fp16x3 chain tile shapes: 128x128 vs 256x128 (KFAC_LP_BIG=6) vs 128x256 (7)
set -e -o pipefail
export TMPDIR=/tmp
for B in "" 6 7; do
  KFAC_LP_BIG=$B PGEMM_CFGS= timeout -k 10 120 python -u scripts/probes/probe_pgemm.py fp16x3 > gpurun_out/r6_pgemm_fp16x3_big$B.log 2>&1
done
KFAC_LP_BIG=6 timeout -k 10 300 python -u -m pytest tests/test_gpu_precond_fused.py -k "fp16x3" "tests/test_gpu_resnet50_parity.py::test_fused_chain_precision_resnet50_shapes" -x -q -s --timeout 200 --timeout-method thread > gpurun_out/r6_lp_big_tests.log 2>&1
KFAC_LP_BIG=7 timeout -k 10 300 python -u -m pytest tests/test_gpu_precond_fused.py -k "fp16x3" -x -q --timeout 200 --timeout-method thread >> gpurun_out/r6_lp_big_tests.log 2>&1
