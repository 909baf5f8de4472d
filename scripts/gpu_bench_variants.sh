#!/bin/bash
# Durable bench variants with the runner trace: each line of VARIANTS is "name|ENV=V ...|bench args".
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${1:-variants}"
mkdir -p "$O" && cd "$R" && export TMPDIR=/tmp
while IFS='|' read -r name envs args; do
  [ -z "$name" ] && continue
  env SW_RUNNER_TRACE=1 $envs timeout -k 10 200 python -u bench.py --steps ${STEPS:-100} --warmup 10 $args > "$O/$name.log" 2>&1 || exit 1
  tail -1 "$O/$name.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); t=d["detail"].get("runner_trace_ms_per_step",{}); print(sys.argv[1], round(d["value"]/1e6,1),"M/s", d["ms_per_step"], "ms | gpu_h2d", t.get("gpu_h2d"), "h2d->end", t.get("gpu_h2d_to_step_end"), "wait", t.get("wait_step"), "router", d["detail"].get("bus",{}).get("router_ms_per_job"))' "$name"
done <<< "${VARIANTS:-base|SW_PIPELINE_DEPTH=2 SW_ROUTE_THREADS=4|
noalt|SW_PIPELINE_DEPTH=2 SW_ROUTE_THREADS=4|--no-alt-ids}"
