set -o pipefail
export TMPDIR=/tmp
KFAC_PROFILE_MARKER=1 timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/p2 -o run --output-format csv -- python3 bench.py --steps 12 --warmup 10 --check-finite --graphs 0 > gpurun_out/nan_prof_nog.log 2>&1 || { tail gpurun_out/nan_prof_nog.log; exit 1; }
grep -c nan gpurun_out/nan_prof_nog.log; grep "^step" gpurun_out/nan_prof_nog.log | head -4
KFAC_PROFILE_MARKER=1 timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/p3 -o run --output-format csv -- python3 bench.py --steps 12 --warmup 10 --check-finite --eigen-solver serial > gpurun_out/nan_prof_serial.log 2>&1 || { tail gpurun_out/nan_prof_serial.log; exit 1; }
grep -c nan gpurun_out/nan_prof_serial.log; grep "^step" gpurun_out/nan_prof_serial.log | head -4
