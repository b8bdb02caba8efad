#!/bin/bash
# round 3 closing validation: full GPU suite, smoke, driver bench, window
# profile, then the multi-rank rehearsal (gloo ranks sharing the one GPU)
set -o pipefail
bash scripts/gpu_final.sh || exit 1
bash scripts/gpu_r3_rehearse.sh
