set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_resnet50_parity.py -m gpu -x -v --durations=0 --timeout 360 --timeout-method thread > gpurun_out/pytest_parity.log 2>&1; echo "rc=$?" >> gpurun_out/pytest_parity.log; tail -4 gpurun_out/pytest_parity.log
timeout -k 10 300 python -u scripts/bench_reference.py --steps 20 --warmup 5 --ref-tar ref_snapshot/kfac_reference.tar > gpurun_out/ref_bench_bf16.log 2>&1; tail -2 gpurun_out/ref_bench_bf16.log
timeout -k 10 200 python -u scripts/bench_reference.py --steps 20 --warmup 5 --no-kfac --ref-tar ref_snapshot/kfac_reference.tar > gpurun_out/ref_bench_sgd.log 2>&1; tail -1 gpurun_out/ref_bench_sgd.log
