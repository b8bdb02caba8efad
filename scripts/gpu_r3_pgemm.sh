#!/bin/bash
# round 3: pgemm numerics tests + ResNet-50 chain timing (bf16x6, fp32)
set -o pipefail
mkdir -p gpurun_out/r3
export PGEMM_CFGS=
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_precond_fused.py tests/test_gpu_resnet50_parity.py tests/test_gpu_eig_dc.py tests/test_gpu_chol.py > gpurun_out/r3/tests_pgemm.log 2>&1; rc=$?
tail -3 gpurun_out/r3/tests_pgemm.log
[ $rc -eq 0 ] || exit $rc
for p in bf16x6 fp32; do
  timeout -k 10 200 python -u scripts/probes/probe_pgemm.py $p > gpurun_out/r3/pgemm_$p.log 2>&1 || { tail -20 gpurun_out/r3/pgemm_$p.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/r3/pgemm_$p.log
done
