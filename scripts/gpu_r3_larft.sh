#!/bin/bash
# round 3: recursive-doubling larft (compact-WY T) -- eigensolver accuracy tests, inverse-update groups
set -o pipefail
mkdir -p gpurun_out/r3
O=gpurun_out/r3
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_eig_dc.py tests/test_gpu_kernels.py > $O/tests_larft.log 2>&1; rc=$?
tail -2 $O/tests_larft.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/probes/probe_eig_resnet50.py default only_big only_rest > $O/eig_groups_larft.log 2>&1 || { tail -20 $O/eig_groups_larft.log; exit 1; }
grep -E "^(default|only)" $O/eig_groups_larft.log
