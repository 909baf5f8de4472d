#!/bin/bash
# Hardware counters of the bench's step kernels: bench.py (5 steps) under rocprofv3 --pmc, one pass
# per counter group, summarised per kernel on the box; the raw counter files are deleted.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r5_pmc_step"
mkdir -p "$O" && cd /tmp && export TMPDIR=/tmp
pass() {
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d "$O/$name" -o run -- \
      python3 "$R/bench.py" --steps 5 --warmup 2 > "$O/$name.out" 2> "$O/$name.err" || return $?
  for k in k_decode_count k_decode_emit k_lookup k_dedup_claim k_persist k_state_p2 k_zone_mask k_seg_encode k_ix_scatter; do
    python3 "$R/scripts/pmc_summary.py" "$O/$name" $k
  done > "$O/$name.jsonl"
  rm -rf "$O/$name"
  cat "$O/$name.jsonl"
}
pass a FETCH_SIZE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAIT_INST_ANY \
  && pass b WRITE_SIZE TCC_HIT_sum TCC_MISS_sum SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT
