#!/bin/bash
# round 3: BN finalize per-channel workgroups + LDS-DMA SYRK variants, then
# the driver bench and its window profile
set -o pipefail
bash scripts/gpu_r3_syrkdma.sh || exit 1
bash scripts/gpu_r3_bn.sh
