set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_precond_fused.py tests/test_gpu_resnet50_parity.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/pg_tests.log 2>&1 && echo tests-ok &&
PGEMM_CFGS= timeout -k 10 200 python3 -u scripts/probes/probe_pgemm.py bf16x6 > gpurun_out/pg_mixed.log 2>&1 &&
KFAC_X6_MODE=fp32 PGEMM_CFGS= timeout -k 10 200 python3 -u scripts/probes/probe_pgemm.py bf16x6 > gpurun_out/pg_fp32.log 2>&1 &&
KFAC_X6_MODE=planes PGEMM_CFGS= timeout -k 10 200 python3 -u scripts/probes/probe_pgemm.py bf16x6 > gpurun_out/pg_planes.log 2>&1; echo rc=$?
