mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/probes/probe_two_stage.py --sizes 200,1000,4608 > gpurun_out/ts.log 2>&1 || { echo probe failed; tail -20 gpurun_out/ts.log; exit 1; }
tail -20 gpurun_out/ts.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ts -o ts -- python3 -u scripts/probes/probe_two_stage.py --sizes 4608 > gpurun_out/prof_ts.log 2>&1 || { echo prof failed; tail -20 gpurun_out/prof_ts.log; exit 1; }
find gpurun_out/prof_ts -name "*kernel_stats.csv" | head -3
