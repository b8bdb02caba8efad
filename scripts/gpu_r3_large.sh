#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_eig_dc.py > gpurun_out/r3/test_eig_dc.log 2>&1; echo "eig tests rc=$?"
tail -3 gpurun_out/r3/test_eig_dc.log
for n in 8256 10000; do
  timeout -k 10 200 python -u scripts/probes/probe_eig_large.py $n > gpurun_out/r3/eig_large_$n.log 2>&1 || { tail -5 gpurun_out/r3/eig_large_$n.log; exit 1; }
  grep -E "^(reduction|divide|full)" gpurun_out/r3/eig_large_$n.log | sed "s/^/n=$n /"
done
timeout -k 10 300 python -u scripts/probes/probe_eig_resnet50.py default only_big only_rest > gpurun_out/r3/eig_groups.log 2>&1 || { tail -20 gpurun_out/r3/eig_groups.log; exit 1; }
grep -E "^(default|only)" gpurun_out/r3/eig_groups.log
bash scripts/prof_run.sh r3_eig 300 -- python scripts/probes/probe_eig_resnet50.py default || exit 1
python - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/prof_r3_eig/*kernel_stats.csv')[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print('total kernel ms %.1f' % (tot / 1e6))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:14]:
    print('%9.2f ms %7s calls %9.2f us  %s' % (float(r['TotalDurationNs']) / 1e6, r['Calls'], float(r['AverageNs']) / 1e3, r['Name'][:90]))
PY
