set -o pipefail
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --steps 100 --warmup 10 --profile-phases > gpurun_out/hwq_$q.log 2>&1 || { tail -5 gpurun_out/hwq_$q.log; exit 1; }
  echo "hwq=$q $(tail -1 gpurun_out/hwq_$q.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kfac_phase_ms_total"])')"
done
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python bench.py --steps 100 --warmup 10 > gpurun_out/hwq_16g.log 2>&1 || exit 1
tail -1 gpurun_out/hwq_16g.log
