#!/bin/bash
# round 3: eigensolver GEMMs (back-transformation, D&C merges) on bf16x6 vs fp32:
# accuracy tests, ResNet-50 inverse-update groups under both
set -o pipefail
mkdir -p gpurun_out/r3
O=gpurun_out/r3
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_eig_dc.py tests/test_gpu_kernels.py tests/test_gpu_resnet50_parity.py tests/test_gpu_kfac.py > $O/tests_eiggemm.log 2>&1; rc=$?
tail -3 $O/tests_eiggemm.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/probes/probe_eig_resnet50.py default only_big only_rest fs3 fs1 > $O/eig_groups_x6.log 2>&1 || { tail -20 $O/eig_groups_x6.log; exit 1; }
grep -E "^(default|only|fs)" $O/eig_groups_x6.log
KFAC_EIG_GEMM=fp32 timeout -k 10 300 python -u scripts/probes/probe_eig_resnet50.py default only_big only_rest > $O/eig_groups_f32.log 2>&1 || { tail -20 $O/eig_groups_f32.log; exit 1; }
grep -E "^(default|only)" $O/eig_groups_f32.log
