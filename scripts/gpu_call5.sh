set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/prof_run.sh ts 300 -- python -u scripts/probes/probe_eig_resnet50.py two_stage_fs1 && tail -3 gpurun_out/prof_ts.log
