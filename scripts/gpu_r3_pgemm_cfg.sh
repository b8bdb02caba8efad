#!/bin/bash
# round 3: pgemm tile-configuration sweep on the ResNet-50 chain (timing + max diff vs default)
set -o pipefail
mkdir -p gpurun_out/r3
for p in bf16x6 fp32; do
  PGEMM_CFGS=${CFGS:-0,8,12,13} timeout -k 10 300 python -u scripts/probes/probe_pgemm.py $p > gpurun_out/r3/pgemm_cfg_$p.log 2>&1 || { tail -20 gpurun_out/r3/pgemm_cfg_$p.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/r3/pgemm_cfg_$p.log
done
