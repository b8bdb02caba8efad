set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_eig_two_stage.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_2s.log 2>&1; echo "rc=$?" >> gpurun_out/pytest_2s.log; tail -15 gpurun_out/pytest_2s.log
timeout -k 10 400 python -u scripts/bench_reference.py --steps 20 --warmup 5 --ref-tar ref_snapshot/kfac_reference.tar > gpurun_out/ref_bench_bf16.log 2>&1; tail -2 gpurun_out/ref_bench_bf16.log
