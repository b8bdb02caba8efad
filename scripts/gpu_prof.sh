#!/bin/bash
# rocprofv3 kernel stats of the headline bench (1 GPU) -> gpurun_out/prof_bench/
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/prof_run.sh bench 400 -- python3 bench.py --steps 100 --warmup 10 || { tail -20 gpurun_out/prof_bench.log; exit 1; }
tail -2 gpurun_out/prof_bench.log
ls gpurun_out/prof_bench
