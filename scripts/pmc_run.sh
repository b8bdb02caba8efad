#!/bin/bash
# usage: scripts/pmc_run.sh <name> <timeout_s> "<counters>" [--filter <regex>] -- <program ...>
# One rocprofv3 PMC pass (kernel dispatch counters only, no traces), summarised
# per kernel into gpurun_out/pmc_<name>.csv (raw per-dispatch CSV dropped).
# A heartbeat line goes to gpurun_out/heartbeat.log every 30 s (rocprofv3 is
# silent until it ends).
name=$1; tmo=$2; ctrs=$3; shift 3
filt=()
if [ "$1" = "--filter" ]; then filt=(--kernel-include-regex "$2"); shift 2; fi
[ "$1" = "--" ] && shift
export TMPDIR=/tmp
rm -rf /tmp/pmc_$name
timeout -s KILL $tmo rocprofv3 --pmc $ctrs "${filt[@]}" -d /tmp/pmc_$name -o run \
  --output-format csv -- "$@" > gpurun_out/pmc_$name.log 2>&1 &
pid=$!
while kill -0 $pid 2>/dev/null; do
  sleep 30
  echo "pmc $name running ${SECONDS}s" >> gpurun_out/heartbeat.log
done
wait $pid
rc=$?
python3 scripts/pmc_summary.py /tmp/pmc_$name gpurun_out/pmc_$name.csv >> gpurun_out/pmc_$name.log 2>&1
echo "pmc rc=$rc" >> gpurun_out/pmc_$name.log
exit $rc
