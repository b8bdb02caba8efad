set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_eig_two_stage.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_2s.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_2s.log
[ $rc -eq 0 ] || exit 1
bash scripts/prof_run.sh ts 300 -- python -u scripts/probes/probe_eig_resnet50.py two_stage && grep -A3 "^factors" gpurun_out/prof_ts.log | head -4
