#!/bin/bash
# Tenant path at one batch size over many batches (steady state, not the commit tail of a short run).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${1:-tenant_long}"
B=${B:-65536}; N=${N:-300}
mkdir -p "$O" && cd "$R" && export TMPDIR=/tmp
for P in ${PS:-0 0.01}; do
  timeout -k 10 500 python -u scripts/bench_tenant_path.py --devices 50000 --batch $B --batches $N --warmup 8 \
    --via-bus --max-msgs ${MAXM:-262144} --p-unregistered $P > "$O/tenant_${B}_${P}_${N}.log" 2>&1 || { tail -20 "$O/tenant_${B}_${P}_${N}.log"; exit 1; }
  tail -1 "$O/tenant_${B}_${P}_${N}.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["batch"], d["p_unregistered"], round(d["events_per_sec"]/1e6,1), "M/s", d["ms_per_batch"], "ms/batch", "steps", d.get("engine_steps"))'
done
