#!/bin/bash
# Compensate parity + the C++ API transcript (repeated: it once differed).
set -o pipefail
OUT=gpurun_out/r2c; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_compensate.py tests/test_gpu_cxx_api.py -v --timeout 120 --timeout-method thread > $OUT/comp.log 2>&1 || { tail -40 $OUT/comp.log; exit 1; }
tail -15 $OUT/comp.log
g++ -O2 -std=gnu++17 -ffp-contract=off -Iinclude -o $OUT/probe tests/cpp/lora_phy_api_probe.cpp -Llora-sdr-lightweight-standalone-library-clean_amd/lib -llora_phy_amd -Wl,-rpath,$PWD/lora-sdr-lightweight-standalone-library-clean_amd/lib
for i in 1 2 3 4 5 6; do timeout -k 10 60 $OUT/probe tests/golden > $OUT/t$i.txt || exit 1; done
timeout -k 10 60 oracle/_ref/lora_phy_api_probe_ref tests/golden > $OUT/ref.txt || exit 1
for i in 1 2 3 4 5 6; do cmp $OUT/t$i.txt $OUT/ref.txt && echo "run $i identical"; done; true
