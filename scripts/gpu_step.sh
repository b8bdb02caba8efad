set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_graphs.py > gpurun_out/t_graphs.log 2>&1
echo rc=$?
