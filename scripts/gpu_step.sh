set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
export MIOPEN_FIND_MODE=FAST
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_x6.log 2>&1 && \
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 --precond-precision fp32 > gpurun_out/bench_f32.log 2>&1 && \
timeout -k 10 400 python3 -u bench.py --steps 100 --warmup 10 > gpurun_out/bench_x6_100.log 2>&1
echo rc=$?
