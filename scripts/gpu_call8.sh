set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 420 --timeout-method thread --durations=25 > gpurun_out/pytest_gpu_full.log 2>&1; echo "rc=$?" >> gpurun_out/pytest_gpu_full.log; tail -32 gpurun_out/pytest_gpu_full.log
