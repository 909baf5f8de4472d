#!/bin/bash
# Durable tenant path at 64K-payload raw records, 1200 batches (78.6M events) per configuration:
# steady-state rate and the timed window's submit-interval tail.  Results under gpurun_out/<name>.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${1:-tenant_long}"
mkdir -p "$O" && cd "$R" && export TMPDIR=/tmp
for CAP in 1048576 262144; do
  SW_TENANT_TRACE=1 timeout -k 10 400 python -u scripts/bench_tenant_path.py --devices 50000 --batch 65536 --batches 1200 \
    --warmup 4 --via-bus --max-msgs $CAP > "$O/tenant_65536_0_1200_cap${CAP}.log" 2>&1 \
    || { tail -20 "$O/tenant_65536_0_1200_cap${CAP}.log"; exit 1; }
  tail -1 "$O/tenant_65536_0_1200_cap${CAP}.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["batch"], round(d["events_per_sec"]/1e6,1), "M/s", d["ms_per_batch"], "ms/batch", d["engine_steps"], "steps", d.get("median_ms_second_half"))'
done
