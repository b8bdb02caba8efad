#!/bin/bash
# Two-stage eigensolver session: GPU tests, stage-2 phase stamps, rocprofv3 stats of the
# ResNet-50 inverse update through the two-stage path (KFAC_EIG_TWO_STAGE variant).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_eig_two_stage.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_2s.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_2s.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u scripts/probes/probe_sb2st_stamps.py 4608 30 > gpurun_out/sb_stamps.log 2>&1; cat gpurun_out/sb_stamps.log | tail -4
bash scripts/prof_run.sh ts 300 -- python -u scripts/probes/probe_eig_resnet50.py two_stage && grep -A2 "^factors" gpurun_out/prof_ts.log | head -3
