#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python scripts/debug_smoke.py serial 0 > gpurun_out/dbg_serial.log 2>&1 || { echo "serial failed rc=$?"; tail -60 gpurun_out/dbg_serial.log; exit 1; }
tail -3 gpurun_out/dbg_serial.log
timeout -k 10 240 python scripts/debug_smoke.py auto 1 > gpurun_out/dbg_auto.log 2>&1 || { echo "auto failed rc=$?"; tail -60 gpurun_out/dbg_auto.log; exit 1; }
tail -3 gpurun_out/dbg_auto.log
