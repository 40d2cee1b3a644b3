#!/bin/bash
# Default bench line + kernel-trace stats + C2 line.  usage: bash tools/gpu_bench_prof.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/bp}; mkdir -p "$OUT"; ROOT=$(pwd)
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cut -c1-600 "$OUT/bench.json"
timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline --steps 20 --warmup 10 > "$OUT/c2.json" 2> "$OUT/c2.err" || { tail -20 "$OUT/c2.err"; exit 1; }
cut -c1-400 "$OUT/c2.json"
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof" -o run --output-format csv -- python3 "$ROOT/bench.py" --no-cpu-baseline > "$ROOT/$OUT/prof.log" 2>&1 || { echo "rocprof failed"; tail "$ROOT/$OUT/prof.log"; exit 1; }
find "$ROOT/$OUT/prof" -name "*kernel_stats.csv" -exec head -8 {} \; | cut -c1-200
