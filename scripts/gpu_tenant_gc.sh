#!/bin/bash
# 64K-payload tenant path at cap 256K, 1200 batches: default collector vs gc.freeze() after set-up
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${1:-tenant_gc}"
mkdir -p "$O" && cd "$R" && export TMPDIR=/tmp
for GC in freeze default; do
  SW_TENANT_TRACE=1 timeout -k 10 400 python -u scripts/bench_tenant_path.py --devices 50000 --batch 65536 --batches 1200 \
    --warmup 4 --via-bus --max-msgs 262144 --gc $GC > "$O/tenant_cap262144_gc_${GC}.log" 2>&1 \
    || { tail -20 "$O/tenant_cap262144_gc_${GC}.log"; exit 1; }
  tail -1 "$O/tenant_cap262144_gc_${GC}.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["gc"], round(d["events_per_sec"]/1e6,1), "M/s", d["ms_per_batch"], "ms/batch", d["engine_steps"], "steps", d["routed_payloads"], "routed", d.get("median_ms_second_half"))'
done
