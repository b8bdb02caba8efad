# Per-column F / S / U times of the one-stage reduction for eigensolver
# grouping variants (probe_eig_resnet50.py <variant>), from kernel traces.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in ${VARIANTS:-fs1 only_big}; do
  rm -rf /tmp/tr_$v
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/tr_$v -o run --output-format csv -- \
    python3 -u scripts/probes/probe_eig_resnet50.py $v > gpurun_out/tr_$v.log 2>&1 || { echo "$v failed"; exit 1; }
  f=$(find /tmp/tr_$v -name "*kernel_trace.csv" | head -1)
  python3 scripts/probes/trace_reduce_columns.py "$f" 4 > gpurun_out/tr_${v}_columns.log 2>&1
  echo "== $v"; grep -v "^/opt" gpurun_out/tr_$v.log | head -3; cat gpurun_out/tr_${v}_columns.log
done
