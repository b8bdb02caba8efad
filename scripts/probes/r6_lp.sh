#!/bin/bash
# Round-6 low-plane chain modes: fused-chain tests (fp16x3, inv_dtype) and the
# ResNet-50 chain timing per precision.  Stops at the first GPU failure.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_precond_fused.py "tests/test_gpu_resnet50_parity.py::test_fused_chain_precision_resnet50_shapes" -x -q -s --timeout 200 --timeout-method thread > gpurun_out/r6_lp_tests.log 2>&1
rc=$?; echo rc=$rc >> gpurun_out/r6_lp_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for P in ${PRECS:-bf16x6 fp16x3}; do
  PGEMM_CFGS= timeout -k 10 120 python -u scripts/probes/probe_pgemm.py $P > gpurun_out/r6_pgemm_$P.log 2>&1 || exit 1
done
