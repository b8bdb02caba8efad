#!/bin/bash
# Round 6: BN finalize folded into the apply pass for small layers -- BN and
# model tests, then the bench with and without the fold on the same box.
set -e -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_bn.py tests/test_gpu_models.py tests/test_gpu_graphs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6_bn_fold_tests.log 2>&1
KFAC_BN_FOLD_M=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6_bench_nofold.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6_bench_fold.log 2>&1
KFAC_BN_FOLD_M=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6_bench_nofold2.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6_bench_fold2.log 2>&1
