#!/bin/bash
# Multi-rank rehearsal of bench.py's distributed path on a ONE-GPU box: N ranks
# share cuda:0 over gloo (RCCL refuses duplicate devices), with the cross-rank
# comm consistency checks on.  The 8-GPU RCCL run is the driver's.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
N=${N:-2}
KFAC_DIST_BACKEND=gloo KFAC_COMM_CHECK=1 timeout -k 10 400 python -m torch.distributed.run \
  --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus $N --steps ${STEPS:-20} --warmup ${WARMUP:-5} ${BENCH_ARGS} \
  > gpurun_out/rehearse_n$N.log 2>&1
rc=$?
echo "rehearsal N=$N rc=$rc" >> gpurun_out/rehearse_n$N.log
grep '"metric"' gpurun_out/rehearse_n$N.log || tail -30 gpurun_out/rehearse_n$N.log
exit $rc
