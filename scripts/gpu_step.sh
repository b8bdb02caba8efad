set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_resnet50_parity.py > gpurun_out/t_parity.log 2>&1
echo rc=$?
