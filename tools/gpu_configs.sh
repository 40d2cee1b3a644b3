#!/bin/bash
# Every BASELINE config's bench line + the perf CSV.  usage: bash tools/gpu_configs.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/cfg}; mkdir -p "$OUT"
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "$n failed"; tail -20 "$OUT/$n.err"; exit 1; }
  cut -c1-300 "$OUT/$n.json"
}
run c1 --csv "$OUT/perf.csv" --run-id "${RUN_ID:-r3}"
run c2 --config c2 --no-cpu-baseline --steps 20 --warmup 10
run c3 --config c3
run c4 --config c4
cat "$OUT/perf.csv"
