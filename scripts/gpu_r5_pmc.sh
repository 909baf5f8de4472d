#!/bin/bash
# k_seg_encode hardware counters: the encoder bench (1M rows with strings) under rocprofv3 --pmc, one
# pass per counter group, summarised on the box; the raw counter files are deleted.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r5_pmc"
mkdir -p "$O" && cd /tmp && export TMPDIR=/tmp
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$O/$name" -o run -- \
      python3 "$R/scripts/bench_seg_encode.py" --n 1048576 --reps 5 > "$O/$name.out" 2> "$O/$name.err" || return $?
  python3 "$R/scripts/pmc_summary.py" "$O/$name" k_seg_encode > "$O/$name.json"
  rm -rf "$O/$name"
  cat "$O/$name.json"
}
pass sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES \
  && pass mem FETCH_SIZE SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE
