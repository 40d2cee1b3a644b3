#!/bin/bash
# PMC passes over an arbitrary python driver (one rocprofv3 run per counter
# group, gfx950 slot limits respected; never combined with tracing).
#   bash tools/pmc_k.sh <outdir> <script.py> [args...]
set -u
OUT=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
SCRIPT=$1; shift
cd /tmp && export TMPDIR=/tmp
mkdir -p "$ROOT/$OUT"
run_pass() {
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" -d "$ROOT/$OUT/$name" -o run --output-format csv \
      -- python3 "$ROOT/$SCRIPT" "${ARGS[@]}" > "$ROOT/$OUT/$name.log" 2>&1
}
ARGS=("$@")
run_pass fetch FETCH_SIZE && \
run_pass write WRITE_SIZE && \
run_pass tcc TCC_HIT_sum TCC_MISS_sum && \
run_pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY && \
run_pass sq2 SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE SQ_INSTS_SMEM
echo "pmc rc=$?"
