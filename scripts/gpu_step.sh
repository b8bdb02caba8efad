set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
export MIOPEN_FIND_MODE=FAST
timeout -k 10 300 python3 -u scripts/probes/probe_eig_resnet50.py default > gpurun_out/eig_leaf.log 2>&1 && \
timeout -k 10 600 python3 -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_eig_dc.py tests/test_gpu_eig_tridiag.py tests/test_gpu_kfac.py tests/test_gpu_graphs.py tests/test_gpu_factor_determinism.py > gpurun_out/t_eig.log 2>&1 && \
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
echo rc=$?
