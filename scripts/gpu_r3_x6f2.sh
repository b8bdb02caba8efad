#!/bin/bash
# round 3: X6F conflict-free split stores (numerics, timing, one PMC pass)
set -o pipefail
mkdir -p gpurun_out/r3
O=gpurun_out/r3
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_precond_fused.py tests/test_gpu_resnet50_parity.py > $O/tests_x6f2.log 2>&1; rc=$?
tail -2 $O/tests_x6f2.log
[ $rc -eq 0 ] || exit $rc
export PGEMM_CFGS=
timeout -k 10 200 python -u scripts/probes/probe_pgemm.py bf16x6 > $O/pgemm_x6f2.log 2>&1 || { tail -20 $O/pgemm_x6f2.log; exit 1; }
grep -v amdgpu.ids $O/pgemm_x6f2.log
bash scripts/pmc_run.sh x6f2a 150 "SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" --filter "pgemm_kernel<3" -- python3 scripts/probes/probe_pgemm.py bf16x6 || exit 1
cat gpurun_out/pmc_x6f2a.csv
