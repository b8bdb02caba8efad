set -e
for d in 0 1 2 3; do
  KFAC_SB2ST_DBG=$d timeout -k 10 120 python -u scripts/probes/probe_two_stage.py --sizes 4608 2>&1 | grep -v amdgpu | grep "ms:" | sed "s/^/dbg=$d /"
done
