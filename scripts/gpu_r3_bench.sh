#!/bin/bash
# round 3: driver bench + phase breakdown of the same config
set -o pipefail
mkdir -p gpurun_out/r3
O=gpurun_out/r3
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { tail -20 $O/bench20.log; exit 1; }
tail -1 $O/bench20.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --profile-phases --sgd-delta 0 > $O/bench20_phases.log 2>&1 || { tail -20 $O/bench20_phases.log; exit 1; }
tail -1 $O/bench20_phases.log
