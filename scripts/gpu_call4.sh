set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_eig_two_stage.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_2s.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/pytest_2s.log; tail -25 gpurun_out/pytest_2s.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u scripts/probes/probe_eig_resnet50.py default two_stage two_stage_fs1 > gpurun_out/probe_2s.log 2>&1; tail -5 gpurun_out/probe_2s.log
