#!/bin/bash
# FETCH_SIZE and WRITE_SIZE passes only (one rocprofv3 --pmc run each, within
# gfx950's TCC limits; never combined with tracing):
#   tools/pmc_fw.sh <outdir> [bench args]      (GPU box, repo root)
set -u
OUT=$1; shift
ARGS=${*:-"--config c2 --steps 2 --warmup 1 --no-cpu-baseline --no-mode-a"}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
mkdir -p "$ROOT/$OUT"
run_pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$ROOT/$OUT/$name" -o run --output-format csv \
      -- python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/$name.log" 2>&1
}
run_pass fetch FETCH_SIZE && run_pass write WRITE_SIZE
echo "pmc rc=$?"
