#!/bin/bash
# usage: scripts/prof_run.sh <outname> <timeout_s> -- python ... ; keeps only the rocprofv3 *stats* CSVs
name=$1; tmo=$2; shift 2; [ "$1" = "--" ] && shift
export TMPDIR=/tmp
out=gpurun_out/prof_$name
rm -rf /tmp/prof_$name
timeout -k 10 $tmo rocprofv3 --kernel-trace --stats -d /tmp/prof_$name -o run --output-format csv -- "$@" > gpurun_out/prof_$name.log 2>&1
rc=$?
mkdir -p $out
find /tmp/prof_$name -name "*stats*.csv" -exec cp {} $out/ \;
echo "rocprof rc=$rc" >> gpurun_out/prof_$name.log
exit $rc
