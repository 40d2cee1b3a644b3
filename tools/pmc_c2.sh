#!/bin/bash
# PMC counters of the C2 workload (SF12 x 4,096 frames, mode 2), one rocprofv3
# pass per counter group within gfx950's per-block limits (<= 8 SQ, FETCH_SIZE
# and WRITE_SIZE in passes of their own); never combined with tracing.
#   tools/pmc_c2.sh <outdir> [bench args]      (GPU box, repo root)
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
run_pass act SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAIT_ANY SQ_WAIT_INST_ANY && \
run_pass ins SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_SALU && \
run_pass lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VMEM_TA_ADDR_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_BUSY_CYCLES && \
run_pass fetch FETCH_SIZE && \
run_pass write WRITE_SIZE
echo "pmc rc=$?"
