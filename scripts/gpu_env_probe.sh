#!/bin/bash
# Runtime-knob probe on the driver's bench command: HIP kernel-argument
# placement (the reduction chain is ~9k dependent launches per inverse step).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in unset 1 0; do
  if [ $v = unset ]; then
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/env_kernarg_$v.log 2>&1 || exit 1
  else
    HIP_FORCE_DEV_KERNARG=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/env_kernarg_$v.log 2>&1 || exit 1
  fi
  echo "kernarg=$v $(tail -1 gpurun_out/env_kernarg_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["step_ms_by_kind"], d["sgd_only_ms_per_step"])')"
done
