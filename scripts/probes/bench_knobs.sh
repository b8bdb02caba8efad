set -o pipefail
mkdir -p gpurun_out
for cfg in "1 1 0" "0 1 0" "0 0 0" "0 1 1" "1 0 0"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --graphs $1 --early-factors $2 --overlap-precond $3 > gpurun_out/b_$1$2$3.log 2>&1 || { echo "bench $cfg failed"; tail -5 gpurun_out/b_$1$2$3.log; exit 1; }
  echo "graphs=$1 early=$2 overlap=$3: $(grep '"metric"' gpurun_out/b_$1$2$3.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r.get("kfac_step_ms",{}).get("by_kind"))')"
done
