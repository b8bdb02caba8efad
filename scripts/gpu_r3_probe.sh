#!/bin/bash
# round 3: eigensolver tests, reduction phase stamps, ResNet-50 inverse-update wall time
set -o pipefail
mkdir -p gpurun_out/r3
O=gpurun_out/r3
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_eig_dc.py > $O/test_eig_dc.log 2>&1; echo "eig tests rc=$?"
tail -4 $O/test_eig_dc.log
timeout -k 10 120 python -u scripts/probes/probe_eig_large.py 10000 > $O/eig_large_10000.log 2>&1 || { tail -20 $O/eig_large_10000.log; exit 1; }
cat $O/eig_large_10000.log
for nb in "4608 1" "1152 1" "4608 3"; do
  set -- $nb
  STAMPS=1 REPS=3 timeout -k 10 120 python -u scripts/probes/probe_reduce_one.py $1 $2 graph > $O/stamps_${1}x${2}.log 2>&1 || { tail -20 $O/stamps_${1}x${2}.log; exit 1; }
  tail -5 $O/stamps_${1}x${2}.log
done
timeout -k 10 300 python -u scripts/probes/probe_eig_resnet50.py default only_big only_rest > $O/eig_groups.log 2>&1 || { tail -20 $O/eig_groups.log; exit 1; }
grep -E "^(default|only)" $O/eig_groups.log
