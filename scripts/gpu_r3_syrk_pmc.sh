#!/bin/bash
# round 3: PMC passes over the grouped factor SYRK (ResNet-50 factor step probe)
set -o pipefail
mkdir -p gpurun_out/r3
bash scripts/pmc_run.sh syrka 150 "SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" --filter "syrk_vec_grouped" -- python3 scripts/probes/probe_factors.py || exit 1
bash scripts/pmc_run.sh syrkb 150 "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_INSTS_SALU TCC_HIT_sum TCC_MISS_sum" --filter "syrk_vec_grouped" -- python3 scripts/probes/probe_factors.py || exit 1
cat gpurun_out/pmc_syrka.csv gpurun_out/pmc_syrkb.csv
