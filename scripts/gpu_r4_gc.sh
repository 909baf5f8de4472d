#!/bin/bash
# Alternate-id tenant path (64K records, cap 256K, 1200 batches) with the collector frozen after
# setup: are the 200+ ms submit stalls Python GC pauses?
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/tenant_gc"
mkdir -p "$O" && cd "$R" && export TMPDIR=/tmp
SW_TENANT_TRACE=1 timeout -k 10 400 python -u scripts/bench_tenant_path.py --devices 50000 --batch 65536 --batches 1200 \
  --warmup 4 --via-bus --max-msgs 262144 --gc freeze > "$O/alt_gc_freeze.log" 2> "$O/alt_gc_freeze.err" || exit $?
tail -1 "$O/alt_gc_freeze.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["events_per_sec"]/1e6,1), "M/s", d["mean_ms"], d.get("median_ms_second_half"))'
