#!/bin/bash
# Durable tenant path (gpu-columnar) at 64K-payload raw records, 300-batch steady state with
# coalescing, traced (per-batch host stages).  Results under gpurun_out/<name>.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${1:-r4_tenant}"
mkdir -p "$O" && cd "$R" && export TMPDIR=/tmp
for CFG in "1048576 0" "1048576 0.01" "262144 0"; do
  set -- $CFG
  CAP=$1; P=$2
  SW_TENANT_TRACE=1 timeout -k 10 300 python -u scripts/bench_tenant_path.py --devices 50000 --batch 65536 --batches 300 \
    --warmup 4 --via-bus --max-msgs $CAP --p-unregistered $P > "$O/tenant_65536_${P}_300_cap${CAP}.log" 2>&1 \
    || { tail -20 "$O/tenant_65536_${P}_300_cap${CAP}.log"; exit 1; }
  tail -1 "$O/tenant_65536_${P}_300_cap${CAP}.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["batch"], d["p_unregistered"], round(d["events_per_sec"]/1e6,1), "M/s", d["ms_per_batch"], "ms/batch", d["engine_steps"], "steps", d.get("median_ms_second_half"))'
done
