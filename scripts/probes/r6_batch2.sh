#!/bin/bash
# Round 6: fp16x3 tile shapes (r6_lp_big.sh), then the inverse-share
# projection / BATCHED_COST_MS refit on the current solver.
set -e -o pipefail
export TMPDIR=/tmp
bash scripts/probes/r6_lp_big.sh
timeout -k 10 500 python -u scripts/probes/probe_inverse_share.py > gpurun_out/r6_inverse_share.log 2>&1
