#!/bin/bash
# List (default) or terminate THIS USER's processes that hold an AMD GPU
# (reference: scripts/kill_python_process.sh, which parsed nvidia-smi and
# kill -9'd every python process).  Only exact PIDs owned by the caller are
# touched -- never a name pattern.  Usage: kill_gpu_processes.sh [--kill]
set -euo pipefail
pids=$(rocm-smi --showpids 2>/dev/null | awk '/^[0-9]+/{print $1}' | sort -u || true)
mine=()
for p in $pids; do
  if [ "$(stat -c %U /proc/$p 2>/dev/null || true)" = "$(id -un)" ]; then mine+=("$p"); fi
done
if [ ${#mine[@]} -eq 0 ]; then echo "no GPU processes of $(id -un)"; exit 0; fi
printf 'GPU processes of %s: %s\n' "$(id -un)" "${mine[*]}"
if [ "${1:-}" = "--kill" ]; then kill -TERM "${mine[@]}"; echo "sent SIGTERM"; fi
