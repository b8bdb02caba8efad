set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
export MIOPEN_FIND_MODE=FAST
timeout -k 10 400 python3 -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_bn.py tests/test_gpu_models.py tests/test_gpu_graphs.py tests/test_gpu_kfac.py > gpurun_out/t_bn.log 2>&1; echo "rc=$?" >> gpurun_out/t_bn.log
