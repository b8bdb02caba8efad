set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_eig_dc.py > gpurun_out/t_dc.log 2>&1 && \
for k in 2 3 4; do KFAC_EIG_FUSED_STREAMS=$k timeout -k 10 200 python3 -u scripts/probes/probe_eig_resnet50.py default > gpurun_out/eig_s$k.log 2>&1 || exit 1; done
echo rc=$?
