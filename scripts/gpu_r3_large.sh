#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r3
for n in 8256 8320 10000 16384; do
  timeout -k 10 200 python -u scripts/probes/probe_eig_large.py $n > gpurun_out/r3/eig_large_$n.log 2>&1 || { tail -5 gpurun_out/r3/eig_large_$n.log; exit 1; }
  grep -E "^(reduction|divide|full)" gpurun_out/r3/eig_large_$n.log | sed "s/^/n=$n /"
done
