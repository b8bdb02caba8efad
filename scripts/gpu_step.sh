set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
export MIOPEN_FIND_MODE=FAST
N=2 STEPS=12 WARMUP=3 bash scripts/gpu_rehearse_multirank.sh
echo rc=$?
