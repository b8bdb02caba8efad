#!/bin/bash
# rocprofv3 hardware-counter passes over one ResNet-50 K-FAC step (factor SYRK,
# every eigensolver path, fused preconditioning chain): scripts/probes/probe_pgemm.py.
# One pass per counter group (block limits: 8 SQ, 4 TCC), each under its own
# kill timeout; summaries -> gpurun_out/pmc/.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
pass() {  # pass <name> <counters...>
  local name=$1; shift
  rm -rf /tmp/$name
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc "$@" -d /tmp/$name -o run --output-format csv \
    -- python3 scripts/probes/probe_pgemm.py bf16x3 > gpurun_out/pmc/$name.log 2>&1 || {
      echo "$name failed"; tail -5 gpurun_out/pmc/$name.log; exit 1; }
  f=$(find /tmp/$name -name "*counter_collection.csv" | head -1)
  cp "$f" /tmp/$name.csv
  echo "$name ok"
}
pass pmc1 SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
pass pmc2 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F32 GRBM_GUI_ACTIVE FETCH_SIZE
pass pmc3 TCC_HIT_sum TCC_MISS_sum WRITE_SIZE
python3 scripts/pmc_summary.py /tmp/pmc1.csv /tmp/pmc2.csv /tmp/pmc3.csv > gpurun_out/pmc/summary.txt
head -c 300 /tmp/pmc1.csv > gpurun_out/pmc/csv_header.txt
cat gpurun_out/pmc/summary.txt
