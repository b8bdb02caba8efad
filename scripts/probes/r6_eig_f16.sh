#!/bin/bash
# Round 6: eigensolver GEMMs with bounded operands on fp16x3 (PREC_F16X3F):
# eigensolver / parity tests, then D&C + back-transformation and the ResNet-50
# inverse update against KFAC_EIG_GEMM=bf16x6 on the same box.
set -e -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_eig_dc.py tests/test_gpu_resnet50_parity.py tests/test_gpu_kfac.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6_eig_f16_tests.log 2>&1
for G in bf16x6 f16x3; do
  KFAC_EIG_GEMM=$G timeout -k 10 200 python -u scripts/probes/probe_reduce.py > gpurun_out/r6_eig_gemm_$G.log 2>&1
  KFAC_EIG_GEMM=$G timeout -k 10 200 python -u scripts/probes/probe_eig_resnet50.py default only_big only_rest > gpurun_out/r6_eig50_gemm_$G.log 2>&1
done
