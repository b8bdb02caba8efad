#!/bin/bash
# round 3: PMC passes over the bf16x6 fp32-operand chain (pgemm_kernel<3,...>)
set -o pipefail
mkdir -p gpurun_out/r3
export PGEMM_CFGS=
bash scripts/pmc_run.sh x6fa 150 "SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU" --filter "pgemm_kernel<3" -- python3 scripts/probes/probe_pgemm.py bf16x6 || exit 1
bash scripts/pmc_run.sh x6fb 150 "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_ACTIVE_INST_MISC TCC_HIT_sum TCC_MISS_sum" --filter "pgemm_kernel<3" -- python3 scripts/probes/probe_pgemm.py bf16x6 || exit 1
bash scripts/pmc_run.sh x6fc 150 "FETCH_SIZE" --filter "pgemm_kernel<3" -- python3 scripts/probes/probe_pgemm.py bf16x6 || exit 1
cat gpurun_out/pmc_x6fa.csv gpurun_out/pmc_x6fb.csv gpurun_out/pmc_x6fc.csv
