#!/bin/bash
# The round-end driver's bench command (explicit --steps 20 --warmup 5), run twice.
set -o pipefail
OUT=${1:-gpurun_out/drv}; mkdir -p "$OUT"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/b$i.json" 2> "$OUT/b$i.err" || { tail -20 "$OUT/b$i.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/b$i.json'));print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['stage_ms'])"
done
