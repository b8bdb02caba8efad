# Kernel trace of the bench's timed window + idle-gap analysis.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf /tmp/prof_gaps
KFAC_PROFILE_MARKER=1 timeout -k 10 600 rocprofv3 --kernel-trace -d /tmp/prof_gaps -o run \
  --output-format csv -- python3 bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-5} $BENCH_ARGS > gpurun_out/gaps_bench.log 2>&1 || exit 1
f=$(find /tmp/prof_gaps -name "*kernel_trace.csv" | head -1)
python3 scripts/probes/trace_gaps.py "$f" 20 > gpurun_out/gaps.txt
python3 scripts/prof_window.py "$f" ${STEPS:-20} > gpurun_out/gaps_window.txt
head -60 gpurun_out/gaps.txt
