#!/bin/bash
# round 3: grouped factor launches from the last gradient hook
# (compute_factor_in_hook=True, the multi-rank mode): bitwise tests, graph tests,
# probe of the factor-step cost, multi-rank gloo rehearsal
set -o pipefail
mkdir -p gpurun_out/r3
O=gpurun_out/r3
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_factor_determinism.py tests/test_gpu_graphs.py tests/test_gpu_mixed.py tests/test_gpu_examples.py tests/test_gpu_overlap_precond.py > $O/tests_hookgrp.log 2>&1; rc=$?
tail -2 $O/tests_hookgrp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 250 python -u scripts/probes/probe_hook_factors.py > $O/hook_factors.log 2>&1 || { tail -20 $O/hook_factors.log; exit 1; }
grep -v amdgpu $O/hook_factors.log
bash scripts/gpu_r3_rehearse.sh
