#!/bin/bash
# usage: scripts/pmc_run.sh <name> <timeout_s> "<counters>" -- <program ...>
# One rocprofv3 PMC pass (kernel dispatch counters only, no traces), summarised
# per kernel into gpurun_out/pmc_<name>.csv (raw per-dispatch CSV dropped).
name=$1; tmo=$2; ctrs=$3; shift 3; [ "$1" = "--" ] && shift
export TMPDIR=/tmp
rm -rf /tmp/pmc_$name
timeout -s KILL $tmo rocprofv3 --pmc $ctrs -d /tmp/pmc_$name -o run --output-format csv -- "$@" \
  > gpurun_out/pmc_$name.log 2>&1
rc=$?
python3 scripts/pmc_summary.py /tmp/pmc_$name gpurun_out/pmc_$name.csv >> gpurun_out/pmc_$name.log 2>&1
echo "pmc rc=$rc" >> gpurun_out/pmc_$name.log
exit $rc
