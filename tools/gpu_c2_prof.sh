#!/bin/bash
# C2 (SF12 x 4,096) bench line + rocprofv3 kernel stats of the same command.
# usage: bash tools/gpu_c2_prof.sh <outdir> [extra bench args]
set -o pipefail
OUT=${1:-gpurun_out/c2}; shift; mkdir -p "$OUT"; ROOT=$(pwd)
timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline --steps 20 --warmup 10 "$@" > "$OUT/c2.json" 2> "$OUT/c2.err" || { tail -20 "$OUT/c2.err"; exit 1; }
cut -c1-700 "$OUT/c2.json"
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof" -o run --output-format csv -- python3 "$ROOT/bench.py" --config c2 --no-cpu-baseline --no-mode-a --steps 10 --warmup 5 "$@" > "$ROOT/$OUT/prof.log" 2>&1 || { echo "rocprof failed"; tail "$ROOT/$OUT/prof.log"; exit 1; }
find "$ROOT/$OUT/prof" -name "*kernel_stats.csv" -exec cut -c1-220 {} \; | head -14
