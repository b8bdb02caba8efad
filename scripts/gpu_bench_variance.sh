set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench20_rep$i.log 2>&1 && tail -1 gpurun_out/bench20_rep$i.log | cut -c1-200 || exit 1; done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --precond-precision fp32 > gpurun_out/bench20_fp32.log 2>&1 && tail -1 gpurun_out/bench20_fp32.log | cut -c1-200
