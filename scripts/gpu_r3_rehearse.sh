#!/bin/bash
# round 3: multi-rank bench rehearsal on one GPU (gloo): bf16 weights + split-backward
# all-reduce + deferred factor all-reduce; with and without the comm checks
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
run() {  # name N env...
  local name=$1 n=$2; shift 2
  env "$@" KFAC_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus $n --steps 20 --warmup 5 ${BENCH_ARGS} > gpurun_out/r3/rehearse_$name.log 2>&1
  local rc=$?
  echo "rehearsal $name rc=$rc"
  grep '"metric"' gpurun_out/r3/rehearse_$name.log | cut -c1-400 || tail -30 gpurun_out/r3/rehearse_$name.log
  return $rc
}
run n2_check 2 KFAC_COMM_CHECK=1 &&
run n2_graphs 2 KFAC_COMM_CHECK=0 &&
BENCH_ARGS="--comm-method hybrid-opt --grad-worker-fraction 0.5" run n4_hybrid_check 4 KFAC_COMM_CHECK=1
