#!/bin/bash
# round 3: bf16x6 on fp32 operands (in-kernel plane split): numerics tests,
# chain timing vs the plane-stored operands, inverse-step breakdown, bench
set -o pipefail
mkdir -p gpurun_out/r3
O=gpurun_out/r3
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_precond_fused.py tests/test_gpu_resnet50_parity.py tests/test_gpu_overlap_precond.py tests/test_gpu_graphs.py > $O/tests_x6f.log 2>&1; rc=$?
tail -3 $O/tests_x6f.log
[ $rc -eq 0 ] || exit $rc
export PGEMM_CFGS=0,8,9
timeout -k 10 200 python -u scripts/probes/probe_pgemm.py bf16x6 > $O/pgemm_x6f.log 2>&1 || { tail -20 $O/pgemm_x6f.log; exit 1; }
grep -v amdgpu.ids $O/pgemm_x6f.log
KFAC_X6_PLANES=1 timeout -k 10 200 python -u scripts/probes/probe_pgemm.py bf16x6 > $O/pgemm_x6planes.log 2>&1 || { tail -20 $O/pgemm_x6planes.log; exit 1; }
grep -v amdgpu.ids $O/pgemm_x6planes.log
timeout -k 10 300 python -u scripts/probes/probe_inverse_step.py > $O/inverse_step.log 2>&1 || { tail -20 $O/inverse_step.log; exit 1; }
grep -v amdgpu.ids $O/inverse_step.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench20_x6f.log 2>&1 || { tail -20 $O/bench20_x6f.log; exit 1; }
tail -1 $O/bench20_x6f.log
