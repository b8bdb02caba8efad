set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_LDS -d /tmp/pmc1 -o run --output-format csv -- python3 scripts/probes/probe_pgemm.py bf16x3 > gpurun_out/pmc/run1.log 2>&1 || { tail gpurun_out/pmc/run1.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA -d /tmp/pmc2 -o run --output-format csv -- python3 scripts/probes/probe_pgemm.py bf16x3 > gpurun_out/pmc/run2.log 2>&1 || { tail gpurun_out/pmc/run2.log; exit 1; }
for d in pmc1 pmc2; do f=$(find /tmp/$d -name "*counter_collection.csv" | head -1); cp "$f" gpurun_out/pmc/$d.csv; done
ls -la gpurun_out/pmc
