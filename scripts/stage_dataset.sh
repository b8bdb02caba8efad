#!/bin/bash
# Copy a dataset tarball to node-local storage and unpack it once per node
# (reference: scripts/cp_imagenet_to_temp.sh).  Usage: stage_dataset.sh SRC.tar DEST_DIR
set -euo pipefail
SRC=$1; DEST=${2:-/tmp/dataset}
if [ -f "$DEST/.staged" ]; then echo "already staged in $DEST"; exit 0; fi
mkdir -p "$DEST"
tar -xf "$SRC" -C "$DEST"
touch "$DEST/.staged"
echo "staged $SRC -> $DEST"
