#!/bin/bash
# Round-6 reduction sweeps: eigensolver tests, then the single-launch tail
# (KFAC_REDUCE_TAIL) and write-through panel stores (KFAC_REDUCE_UPD_WT)
# against the per-class probe and the ResNet-50 factor set.  One GPU step per
# line, each under its own time limit; stops at the first failure.
set -e -o pipefail
export TMPDIR=/tmp
P=${PFX:-r6_wt}
timeout -k 10 300 python -u -m pytest tests/test_gpu_eig_dc.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${P}_eig_tests.log 2>&1
KFAC_REDUCE_UPD_WT=0 KFAC_REDUCE_TAIL=0 timeout -k 10 200 python -u scripts/probes/probe_reduce.py > gpurun_out/${P}_reduce_base.log 2>&1
for T in ${TAILS_R:-0 1024 2048}; do
  KFAC_REDUCE_TAIL=$T timeout -k 10 200 python -u scripts/probes/probe_reduce.py > gpurun_out/${P}_reduce_tail$T.log 2>&1
done
for T in ${TAILS_E:-0 768 1024 1536}; do
  KFAC_REDUCE_TAIL=$T timeout -k 10 200 python -u scripts/probes/probe_eig_resnet50.py default only_big only_rest > gpurun_out/${P}_eig50_tail$T.log 2>&1
done
