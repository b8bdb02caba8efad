#!/bin/bash
# round 3: SYRK gather through global-address-space loads (no flat loads in
# the k-loop): factor tests, graph tests, factor-step time, PMC pass
set -o pipefail
mkdir -p gpurun_out/r3
O=gpurun_out/r3
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_precond_fused.py tests/test_gpu_factor_determinism.py tests/test_gpu_kernels.py tests/test_gpu_graphs.py tests/test_gpu_mixed.py > $O/tests_syrk_g.log 2>&1; rc=$?
tail -3 $O/tests_syrk_g.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/probes/probe_factors.py > $O/factors_g.log 2>&1 || { tail -20 $O/factors_g.log; exit 1; }
grep -v amdgpu.ids $O/factors_g.log
bash scripts/pmc_run.sh syrkga 150 "SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" --filter "syrk_vec_grouped" -- python3 scripts/probes/probe_factors.py || exit 1
cat gpurun_out/pmc_syrkga.csv
