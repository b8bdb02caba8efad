#!/bin/bash
# Race-detection leg: the GPU kernel + K-FAC tests with every
# kernel launch and copy serialised by the HIP runtime.  A test that passes
# normally but fails here (or the reverse) points at a missing stream/event
# dependency between our side streams (eigensolver workers, lagged inverses,
# graph replays) and the compute stream.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
AMD_SERIALIZE_KERNEL=3 AMD_SERIALIZE_COPY=3 timeout -k 10 600 python -u -m pytest -x -q \
  --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_gpu_kfac.py tests/test_gpu_eig_dc.py \
  tests/test_gpu_graphs.py > gpurun_out/pytest_gpu_serialized.log 2>&1
rc=$?
echo "serialized rc=$rc" >> gpurun_out/pytest_gpu_serialized.log
tail -3 gpurun_out/pytest_gpu_serialized.log
exit $rc
