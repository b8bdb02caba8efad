set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
export REPS=1
P="python3 scripts/probes/probe_reduce_one.py 2304 1"
bash scripts/pmc_run.sh lat_a 90 "SQ_INSTS_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAVES SQ_INSTS_LDS" -- $P && \
bash scripts/pmc_run.sh lat_b 90 "SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" -- $P
echo rc=$?
