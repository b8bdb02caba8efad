#!/bin/bash
# rocprofv3 kernel trace of the headline bench timed window -> gpurun_out/prof_bench/
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_bench
rm -rf /tmp/prof_bench
STEPS=${STEPS:-100}
KFAC_PROFILE_MARKER=1 timeout -k 10 500 rocprofv3 --kernel-trace -d /tmp/prof_bench -o run --output-format csv -- python3 bench.py --steps $STEPS --warmup 10 ${BENCH_ARGS} > gpurun_out/prof_bench.log 2>&1 || { tail -20 gpurun_out/prof_bench.log; exit 1; }
f=$(find /tmp/prof_bench -name "*kernel_trace.csv" | head -1)
python3 scripts/prof_window.py "$f" $STEPS > gpurun_out/prof_bench/window_summary.txt
grep '"metric"' gpurun_out/prof_bench.log | tail -1
cat gpurun_out/prof_bench/window_summary.txt
