set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_eig_dc.py > gpurun_out/t_dc.log 2>&1 && \
timeout -k 10 200 python3 -u scripts/probes/probe_eig_resnet50.py default > gpurun_out/eig.log 2>&1
echo rc=$?
