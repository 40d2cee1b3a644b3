#!/bin/bash
# PMC counters of the kbench kernels (one pass per group, gfx950 limits).
#   tools/pmc_k.sh <outdir> [kbench args]
set -u
OUT=$1; shift
ARGS=${*:-"--sf 7 --frames 65536 --modes 2 --reps 2"}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
mkdir -p "$ROOT/$OUT"
run_pass() {
  local name=$1; shift
  timeout -k 10 120 rocprofv3 --pmc "$@" -d "$ROOT/$OUT/$name" -o run --output-format csv \
      -- python3 "$ROOT/tools/kbench.py" $ARGS > "$ROOT/$OUT/$name.log" 2>&1
}
run_pass lds SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES && \
run_pass wait SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES GRBM_GUI_ACTIVE && \
run_pass fetch FETCH_SIZE && \
run_pass write WRITE_SIZE
echo "pmc rc=$?"
