#!/bin/bash
# round 3: language models on one GPU -- the Transformer LM with its 10k-vocabulary
# head preconditioned (a 10000 x 10000 G factor on the hand-written eigensolver)
# and skipped; the LSTM LM (reference config); bf16x6 preconditioning
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python -u scripts/bench_lm.py "$@" > gpurun_out/r3/lm_$name.log 2>&1
  local rc=$?; tail -1 gpurun_out/r3/lm_$name.log
  return $rc
}
run tfm_head_graphs --impl ours --model transformer --graphs 1 --skip-head 0 --precond-precision bf16x6 &&
run tfm_graphs --impl ours --model transformer --graphs 1 --precond-precision bf16x6 &&
run lstm_graphs --impl ours --graphs 1 --precond-precision bf16x6
