#!/bin/bash
# Single-frame latency of the lora_phy:: drop-in (GPU) beside the reference
# CPU build, per tests/cpp/latency_probe.cpp (the reference perf harness's
# one-call-per-packet loop, rx_runner's chain, the legacy receive chain).
# usage (GPU box, repo root): bash tools/latency.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/lat}; mkdir -p "$OUT"
g++ -O2 -std=gnu++17 -Iinclude -o "$OUT/latency_probe_amd" tests/cpp/latency_probe.cpp \
    -Llora-sdr-lightweight-standalone-library-clean_amd/lib -llora_phy_amd \
    -Wl,-rpath,$(pwd)/lora-sdr-lightweight-standalone-library-clean_amd/lib || exit 1
timeout -k 10 300 "$OUT/latency_probe_amd" 7 12 400 > "$OUT/latency_amd.jsonl" || { echo "drop-in latency failed"; exit 1; }
timeout -k 10 300 oracle/_ref/latency_probe_ref 7 12 400 > "$OUT/latency_ref.jsonl" || { echo "reference latency failed"; exit 1; }
paste -d'\n' "$OUT/latency_amd.jsonl" "$OUT/latency_ref.jsonl" | cut -c1-200
