#!/bin/bash
# 64K-payload tenant path with alternate ids (cap 256K, 1200 batches): a clean run, then one under
# the stack sampler
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${1:-tenant_alt2}"
mkdir -p "$O" && cd "$R" && export TMPDIR=/tmp
run() {
  local name=$1; shift
  SW_TENANT_TRACE=1 timeout -k 10 400 python -u scripts/bench_tenant_path.py --devices 50000 --batch 65536 --batches 1200 \
    --warmup 4 --via-bus --max-msgs 262144 "$@" > "$O/$name.log" 2> "$O/$name.err" \
    || { tail -20 "$O/$name.err"; return 1; }
  tail -1 "$O/$name.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["alt_ids"], round(d["events_per_sec"]/1e6,1), "M/s", d["ms_per_batch"], "ms/batch", d["engine_steps"], "steps", d["routed_payloads"], "routed", d["mean_ms"], d.get("median_ms_second_half"))'
}
run alt && { [ -n "$ALT_ONLY" ] || SW_SAMPLE_STACKS=1 run alt_sampled; }
