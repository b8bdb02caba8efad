#!/bin/bash
# One torchrun per node, one process per MI355X (reference: scripts/launch_node_torch_imagenet.sh).
#
#   NNODES=4 NODE_RANK=<this node> MASTER_ADDR=<node 0 address> \
#       scripts/launch_node_torch_imagenet.sh [extra example flags]
#
# NODE_RANK defaults to the MPI/SLURM rank variables when present (the
# reference read MV2_COMM_WORLD_RANK / OMPI_COMM_WORLD_RANK).
set -euo pipefail
NNODES=${NNODES:-${SLURM_NNODES:-1}}
NODE_RANK=${NODE_RANK:-${SLURM_NODEID:-${OMPI_COMM_WORLD_RANK:-${MV2_COMM_WORLD_RANK:-0}}}}
MASTER_ADDR=${MASTER_ADDR:-127.0.0.1}
MASTER_PORT=${MASTER_PORT:-29500}
GPUS=${GPUS_PER_NODE:-8}
export HSA_ENABLE_IPC_MODE_LEGACY=${HSA_ENABLE_IPC_MODE_LEGACY:-0}   # dmabuf IPC for RCCL
export OMP_NUM_THREADS=${OMP_NUM_THREADS:-4}
ROOT=$(cd "$(dirname "$0")/.." && pwd)

KFAC_ARGS="--kfac-update-freq 100 --kfac-cov-update-freq 10 --damping 0.001 \
  --kfac-comm-method comm-opt --lr-decay 25 35 40 45 50 --epochs 55 --batch-size 32"

exec python -m torch.distributed.run --nnodes "$NNODES" --node-rank "$NODE_RANK" \
  --nproc-per-node "$GPUS" --master-addr "$MASTER_ADDR" --master-port "$MASTER_PORT" \
  "$ROOT/examples/torch_imagenet_resnet.py" $KFAC_ARGS "$@"
