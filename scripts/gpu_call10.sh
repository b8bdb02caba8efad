set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/probes/probe_eig_resnet50.py default only_big only_rest only_big_fs1 only_rest_fs1 > gpurun_out/probe_groups.log 2>&1; tail -7 gpurun_out/probe_groups.log
