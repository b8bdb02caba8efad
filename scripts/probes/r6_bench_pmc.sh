#!/bin/bash
# Round 6: training-quality test, driver bench, and two PMC passes over the
# fp16x3 chain (pgemm kernels only).  Stops at the first GPU failure.
set -e -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_training_quality.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/r6_train_quality.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6_bench20.log 2>&1
bash scripts/pmc_run.sh r6_pgemm_f16x3_a 90 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" --filter pgemm_kernel -- python3 scripts/probes/probe_pgemm.py fp16x3
bash scripts/pmc_run.sh r6_pgemm_f16x3_b 90 "GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU" --filter pgemm_kernel -- python3 scripts/probes/probe_pgemm.py fp16x3
