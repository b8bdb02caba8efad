set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_bn.py tests/test_gpu_kfac.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/bn_tests.log 2>&1 && echo tests-ok &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bn_bench_small.log 2>&1 &&
KFAC_BN_SMALL_M=0 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bn_bench_three.log 2>&1 &&
KFAC_BN_SMALL_M=6272 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bn_bench_6272.log 2>&1
for f in small three 6272; do python3 -c "
import json,sys
for l in open('gpurun_out/bn_bench_$f.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$f', d['value'], d['ms_per_step'], d['step_ms_by_kind'], d['sgd_only_ms_per_step'])
"; done
