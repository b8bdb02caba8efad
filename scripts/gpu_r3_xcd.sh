#!/bin/bash
# round 3: XCD-aware workgroup order in the grouped SYRK and pgemm kernels
# (numerics, factor-step and chain timing, eigensolver groups)
set -o pipefail
mkdir -p gpurun_out/r3
O=gpurun_out/r3
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_precond_fused.py tests/test_gpu_factor_determinism.py tests/test_gpu_kernels.py tests/test_gpu_eig_dc.py tests/test_gpu_resnet50_parity.py > $O/tests_xcd.log 2>&1; rc=$?
tail -2 $O/tests_xcd.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/probes/probe_factors.py > $O/factors_xcd.log 2>&1 || { tail -20 $O/factors_xcd.log; exit 1; }
grep -v amdgpu.ids $O/factors_xcd.log
export PGEMM_CFGS=
timeout -k 10 200 python -u scripts/probes/probe_pgemm.py bf16x6 > $O/pgemm_xcd.log 2>&1 || { tail -20 $O/pgemm_xcd.log; exit 1; }
grep -v amdgpu.ids $O/pgemm_xcd.log
timeout -k 10 300 python -u scripts/probes/probe_eig_resnet50.py default > $O/eig_groups_xcd.log 2>&1 || { tail -20 $O/eig_groups_xcd.log; exit 1; }
grep -E "^default" $O/eig_groups_xcd.log
