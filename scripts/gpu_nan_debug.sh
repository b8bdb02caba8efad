set -o pipefail
KFAC_NO_TAIL_GRAPH=1 timeout -k 10 200 python bench.py --steps 12 --warmup 10 --check-finite > gpurun_out/nan_a.log 2>&1 || exit 1
echo "no tail graph: $(grep -c nan gpurun_out/nan_a.log) nan lines"; grep "^step" gpurun_out/nan_a.log | head -4
timeout -k 10 200 python bench.py --steps 12 --warmup 10 --check-finite --precond-precision fp32 > gpurun_out/nan_b.log 2>&1 || exit 1
echo "fp32: $(grep -c nan gpurun_out/nan_b.log) nan lines"
