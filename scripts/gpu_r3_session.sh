#!/bin/bash
# round 3 session: eigensolver + factor determinism tests, large-n probe,
# ResNet-50 inverse-update groups, rocprof of the inverse update
set -o pipefail
mkdir -p gpurun_out/r3
O=gpurun_out/r3
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_eig_dc.py tests/test_gpu_factor_determinism.py > $O/tests_eig_det.log 2>&1; echo "tests rc=$?"
tail -4 $O/tests_eig_det.log
for n in 8256 10000; do
  timeout -k 10 200 python -u scripts/probes/probe_eig_large.py $n > $O/eig_large_$n.log 2>&1 || { tail -5 $O/eig_large_$n.log; exit 1; }
  grep -E "^(reduction|divide|full)" $O/eig_large_$n.log | sed "s/^/n=$n /"
done
STAMPS=1 REPS=3 timeout -k 10 120 python -u scripts/probes/probe_reduce_one.py 4608 3 graph > $O/stamps_4608x3.log 2>&1 || exit 1
tail -4 $O/stamps_4608x3.log
timeout -k 10 300 python -u scripts/probes/probe_eig_resnet50.py default only_big only_rest > $O/eig_groups.log 2>&1 || { tail -20 $O/eig_groups.log; exit 1; }
grep -E "^(default|only)" $O/eig_groups.log
bash scripts/prof_run.sh r3_eig 300 -- python scripts/probes/probe_eig_resnet50.py default || exit 1
python - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/prof_r3_eig/*kernel_stats.csv')[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print('total kernel ms %.1f (4 inverse updates)' % (tot / 1e6))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:14]:
    print('%9.2f ms %7s calls %9.2f us  %s' % (float(r['TotalDurationNs']) / 1e6, r['Calls'], float(r['AverageNs']) / 1e3, r['Name'][:90]))
PY
