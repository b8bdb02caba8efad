#!/bin/bash
# Language-model K-FAC throughput on one GPU, all variants on the same box:
# this framework (eager, and the whole step captured) vs the reference on the
# reference's LSTM LM config, plus the Transformer LM.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python -u scripts/bench_lm.py "$@" > gpurun_out/lm_$name.log 2>&1
  local rc=$?; tail -1 gpurun_out/lm_$name.log
  return $rc
}
REF="--impl reference --ref-tar ref_snapshot/kfac_reference.tar"
run ours_lstm_graphs --impl ours --graphs 1 &&
run ours_lstm_sgd_graphs --impl ours --graphs 1 --no-kfac &&
run ours_lstm --impl ours &&
run ours_lstm_sgd --impl ours --no-kfac &&
run ref_lstm $REF &&
run ref_lstm_sgd $REF --no-kfac &&
run ours_tfm_graphs --impl ours --model transformer --graphs 1 &&
run ours_tfm_sgd_graphs --impl ours --model transformer --graphs 1 --no-kfac &&
run ours_tfm --impl ours --model transformer
