#!/bin/bash
# driver-command bench, then a kernel-trace profile of the same timed window
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench20.log 2>&1 || { tail -20 gpurun_out/bench20.log; exit 1; }
tail -1 gpurun_out/bench20.log
timeout -k 10 300 python -u scripts/probes/probe_eig_resnet50.py default only_big only_rest > gpurun_out/eig_groups.log 2>&1 || { tail -20 gpurun_out/eig_groups.log; exit 1; }
grep -E "^(default|only)" gpurun_out/eig_groups.log
timeout -k 10 400 python -u scripts/probes/probe_inverse_share.py > gpurun_out/inverse_share.log 2>&1 || { tail -20 gpurun_out/inverse_share.log; exit 1; }
grep -E "^(W=|fit)" gpurun_out/inverse_share.log
STEPS=20 bash scripts/gpu_prof.sh > gpurun_out/prof_bench_summary.log 2>&1; rc=$?; tail -30 gpurun_out/prof_bench_summary.log; exit $rc
