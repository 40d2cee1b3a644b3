#!/bin/bash
# PMC counters of the bench's kernels, one rocprofv3 pass per counter group
# (gfx950 slot limits: TCC FETCH_SIZE and WRITE_SIZE in separate passes; never
# combined with sys/runtime tracing).  Run on the GPU box from the repo root:
#   tools/pmc.sh <outdir> [bench args]
# Output: <outdir>/<pass>/run_counter_collection.csv
set -u
OUT=$1; shift
ARGS=${*:-"--steps 2 --warmup 1 --no-cpu-baseline --no-mode-a"}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
mkdir -p "$ROOT/$OUT"
run_pass() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" -d "$ROOT/$OUT/$name" -o run --output-format csv \
      -- python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/$name.log" 2>&1
}
run_pass fetch FETCH_SIZE && \
run_pass write WRITE_SIZE && \
run_pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY && \
run_pass sq2 SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE
echo "pmc rc=$?"
