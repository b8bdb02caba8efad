#!/bin/bash
# round 3: bf16x6 register-split variant (KFAC_X6_MODE=r) vs LDS-split (f): numerics,
# chain timing per tile configuration, PMC passes of both
set -o pipefail
mkdir -p gpurun_out/r3
O=gpurun_out/r3
KFAC_X6_MODE=r timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_precond_fused.py tests/test_gpu_resnet50_parity.py > $O/tests_x6r.log 2>&1; rc=$?
tail -2 $O/tests_x6r.log
[ $rc -eq 0 ] || exit $rc
export PGEMM_CFGS=0,8,3
for mode in f r; do
  KFAC_X6_MODE=$mode timeout -k 10 200 python -u scripts/probes/probe_pgemm.py bf16x6 > $O/pgemm_mode_$mode.log 2>&1 || { tail -20 $O/pgemm_mode_$mode.log; exit 1; }
  echo "mode $mode"; grep -v amdgpu.ids $O/pgemm_mode_$mode.log
done
export PGEMM_CFGS=
for mode in f r; do
  p=3; [ $mode = r ] && p=4
  KFAC_X6_MODE=$mode bash scripts/pmc_run.sh x6${mode}a 150 "SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU" --filter "pgemm_kernel<$p" -- python3 scripts/probes/probe_pgemm.py bf16x6 || exit 1
  KFAC_X6_MODE=$mode bash scripts/pmc_run.sh x6${mode}b 150 "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_ACTIVE_INST_MISC TCC_HIT_sum TCC_MISS_sum" --filter "pgemm_kernel<$p" -- python3 scripts/probes/probe_pgemm.py bf16x6 || exit 1
  cat gpurun_out/pmc_x6${mode}a.csv gpurun_out/pmc_x6${mode}b.csv
done
