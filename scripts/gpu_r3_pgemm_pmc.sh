#!/bin/bash
# round 3: bf16x6 preconditioning chain -- per-stage times + two PMC passes
set -o pipefail
mkdir -p gpurun_out/r3
export PGEMM_CFGS=
timeout -k 10 200 python -u scripts/probes/probe_pgemm.py bf16x6 > gpurun_out/r3/pgemm_bf16x6.log 2>&1 || { tail -20 gpurun_out/r3/pgemm_bf16x6.log; exit 1; }
cat gpurun_out/r3/pgemm_bf16x6.log
bash scripts/pmc_run.sh pg6a 150 "SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT TCC_HIT_sum TCC_MISS_sum" --filter pgemm -- python3 scripts/probes/probe_pgemm.py bf16x6 || exit 1
bash scripts/pmc_run.sh pg6b 150 "FETCH_SIZE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_BUSY_CU_CYCLES SQ_INSTS_MFMA" --filter pgemm -- python3 scripts/probes/probe_pgemm.py bf16x6 || exit 1
cat gpurun_out/pmc_pg6a.csv gpurun_out/pmc_pg6b.csv
