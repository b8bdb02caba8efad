set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_overlap_precond.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_ov.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_ov.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench20.log 2>&1 && tail -1 gpurun_out/bench20.log &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --overlap-precond 0 > gpurun_out/bench20_noov.log 2>&1 && tail -1 gpurun_out/bench20_noov.log &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --overlap-precond 0 --fused-sgd 0 > gpurun_out/bench20_base.log 2>&1 && tail -1 gpurun_out/bench20_base.log
