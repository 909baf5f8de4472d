#!/bin/bash
# Round 5: the gpu-columnar tenant path (64K-payload records, cap 256K, 1200 batches, via the bus)
# with alternate ids, three runs, per-phase submit trace on; then once without alternate ids.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${1:-r5_tenant}"
mkdir -p "$O" && cd "$R" && export TMPDIR=/tmp
run() {
  local name=$1; shift
  SW_TENANT_TRACE=1 SW_FRAMED_TRACE=1 timeout -k 10 300 python -u scripts/bench_tenant_path.py --devices 50000 --batch 65536 \
    --batches 1200 --warmup 4 --via-bus --max-msgs 262144 "$@" > "$O/$name.log" 2> "$O/$name.err" \
    || { tail -20 "$O/$name.err"; return 1; }
  tail -1 "$O/$name.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["alt_ids"], round(d["events_per_sec"]/1e6,1), "M/s", d["ms_per_batch"], "ms/batch", d.get("submit_interval_ms"), d.get("median_ms_second_half"))'
}
if [ -n "$RUNS" ]; then for r in $RUNS; do run $r || exit 1; done; exit 0; fi
run alt1 && run alt2 && run alt3 && run noalt --no-alt-ids
