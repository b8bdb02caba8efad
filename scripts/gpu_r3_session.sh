#!/bin/bash
# round 3 session: eigensolver tests, stamps, ResNet-50 inverse-update groups (2 and 1 streams)
set -o pipefail
mkdir -p gpurun_out/r3
O=gpurun_out/r3
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_eig_dc.py tests/test_gpu_factor_determinism.py > $O/tests_eig_det.log 2>&1; echo "tests rc=$?"
tail -2 $O/tests_eig_det.log
for nb in "4608 1" "4608 3"; do
  set -- $nb
  STAMPS=1 REPS=3 timeout -k 10 120 python -u scripts/probes/probe_reduce_one.py $1 $2 graph > $O/stamps_${1}x${2}.log 2>&1 || { tail -20 $O/stamps_${1}x${2}.log; exit 1; }
  tail -4 $O/stamps_${1}x${2}.log
done
timeout -k 10 300 python -u scripts/probes/probe_eig_resnet50.py default only_big only_rest fs1 > $O/eig_groups.log 2>&1 || { tail -20 $O/eig_groups.log; exit 1; }
grep -E "^(default|only|fs1)" $O/eig_groups.log
