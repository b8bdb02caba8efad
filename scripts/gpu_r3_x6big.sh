#!/bin/bash
# round 3: bf16x6 fp32-operand chain with bigger tiles for the big problems;
# inverse-step breakdown; factor SYRK probe; bench
set -o pipefail
mkdir -p gpurun_out/r3
O=gpurun_out/r3
export PGEMM_CFGS=
for big in "" 1 6 7; do
  KFAC_X6_BIG=$big timeout -k 10 200 python -u scripts/probes/probe_pgemm.py bf16x6 > $O/pgemm_x6big$big.log 2>&1 || { tail -20 $O/pgemm_x6big$big.log; exit 1; }
  echo "X6_BIG=$big"; grep -v amdgpu.ids $O/pgemm_x6big$big.log
done
timeout -k 10 300 python -u scripts/probes/probe_inverse_step.py > $O/inverse_step.log 2>&1 || { tail -20 $O/inverse_step.log; exit 1; }
grep -v amdgpu.ids $O/inverse_step.log
timeout -k 10 300 python -u scripts/probes/probe_factors.py > $O/factors.log 2>&1 || { tail -20 $O/factors.log; exit 1; }
grep -v amdgpu.ids $O/factors.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench20_x6f.log 2>&1 || { tail -20 $O/bench20_x6f.log; exit 1; }
tail -1 $O/bench20_x6f.log
