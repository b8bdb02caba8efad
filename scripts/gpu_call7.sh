set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bn.py tests/test_gpu_resnet50_parity.py -m gpu -x -v --timeout 200 --timeout-method thread --durations=5 > gpurun_out/pytest_bnpar.log 2>&1; echo "rc=$?" >> gpurun_out/pytest_bnpar.log; tail -12 gpurun_out/pytest_bnpar.log
