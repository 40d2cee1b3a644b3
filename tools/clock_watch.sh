#!/bin/bash
# Shader clock and board power while a GPU command runs (the power-limit
# question of DESIGN §4.6): samples `amd-smi metric` every ~0.25 s into
# <out>.smi while `<cmd...>` runs, then stops.
#   bash tools/clock_watch.sh <out> <cmd...>      (GPU box, repo root)
OUT=$1; shift
( while true; do date +%s.%N; timeout 5 amd-smi metric -g 0 -c -p 2>&1; sleep 0.25; done ) > "$OUT.smi" 2>&1 &
W=$!
"$@" > "$OUT.out" 2>&1
rc=$?
kill $W 2>/dev/null; wait $W 2>/dev/null
exit $rc
