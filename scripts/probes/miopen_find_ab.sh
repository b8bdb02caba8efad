# bench.py under MIOpen find modes; each mode's user find-db / perf-db lands
# in gpurun_out/mdb_<name> (fresh per run)
set -o pipefail
run() {
  name=$1; lim=$2; shift 2
  rm -rf gpurun_out/mdb_$name; mkdir -p gpurun_out/mdb_$name
  t0=$(date +%s)
  env MIOPEN_USER_DB_PATH=$PWD/gpurun_out/mdb_$name MIOPEN_CUSTOM_CACHE_DIR=/tmp/mcache_$name "$@" \
    timeout -k 10 $lim python bench.py --steps 20 --warmup 5 > gpurun_out/mf_$name.log 2>&1 || { echo "$name failed rc=$?"; tail -3 gpurun_out/mf_$name.log; exit 1; }
  echo "$name $(grep -o '"value": [0-9.]*' gpurun_out/mf_$name.log | head -1) wall $(( $(date +%s) - t0 ))s"
}
run default 400 A=1
run normal 600 MIOPEN_FIND_MODE=NORMAL
run search 900 MIOPEN_FIND_ENFORCE=SEARCH
