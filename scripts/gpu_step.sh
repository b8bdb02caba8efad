set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_kfac.py tests/test_gpu_precond_fused.py > gpurun_out/t_chol.log 2>&1
echo rc=$?
