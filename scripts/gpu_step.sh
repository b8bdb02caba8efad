set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_eig_dc.py tests/test_gpu_eig_tridiag.py > gpurun_out/t_dc.log 2>&1 && \
timeout -k 10 300 python3 -u scripts/probes/probe_reduce.py > gpurun_out/r_all.log 2>&1 && \
PGEMM_CFGS=0,2,4,6,7,10,1 timeout -k 10 200 python3 -u scripts/probes/probe_pgemm.py fp32 > gpurun_out/pg_fp32_sweep.log 2>&1 && \
PGEMM_CFGS=0,2,4,6,7,10,1 timeout -k 10 200 python3 -u scripts/probes/probe_pgemm.py bf16x3 > gpurun_out/pg_bf16_sweep.log 2>&1
echo rc=$?
