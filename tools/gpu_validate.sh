#!/bin/bash
# GPU validation pass: gpu tests, default bench line, kernel-trace profile.
# usage (on the box, from the repo root): bash tools/gpu_validate.sh <outdir> [pytest -k expr]
set -o pipefail
OUT=${1:-gpurun_out/val}
K=${2:-}
mkdir -p "$OUT"
ROOT=$(pwd)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${K:+-k "$K"} > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json" | cut -c1-400
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 10 --no-cpu-baseline > "$ROOT/$OUT/prof.log" 2>&1 || { echo "rocprof failed"; exit 1; }
head -6 "$ROOT/$OUT/prof/run_kernel_stats.csv" | cut -c1-160
