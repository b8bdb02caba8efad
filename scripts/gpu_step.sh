set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -v --timeout 200 --timeout-method thread "tests/test_gpu_graphs.py::test_fp16_overflow_step_filtered_on_device" "tests/test_gpu_graphs.py::test_fp16_gradscaler_step_captures" > gpurun_out/t_amp.log 2>&1
echo rc=$?
