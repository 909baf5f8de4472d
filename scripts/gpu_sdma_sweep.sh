#!/bin/bash
# Durable bench under runner variants: VARIANTS="name:ENV=V,ENV=V name2:..." (default: pipeline
# depth 1 vs 2, copy engine runtime-chosen vs engine 2).  Results under gpurun_out/<name>.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${1:-sdma_sweep}"
mkdir -p "$O" && cd "$R" && export TMPDIR=/tmp
for v in ${VARIANTS:-d1:SW_PIPELINE_DEPTH=1 d2:SW_PIPELINE_DEPTH=2 d2e2:SW_PIPELINE_DEPTH=2,SW_SDMA_ENGINE=2}; do
  name=${v%%:*}; envs=${v#*:}
  env $(echo "$envs" | tr ',' ' ') SW_RUNNER_TRACE=1 timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 > "$O/$name.log" 2>&1 || exit 1
  tail -1 "$O/$name.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], round(d["value"]/1e6,1),"M/s", d["ms_per_step"], "ms", d["detail"].get("runner_trace_ms_per_step"), d["detail"].get("bus",{}).get("router_ms_per_job"))' $name
done
