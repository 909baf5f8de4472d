#!/bin/bash
# Host phase trace of the durable bench + kernel profile.  Results under gpurun_out/<name>.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${1:-r3_trace}"
mkdir -p "$O/prof" && cd "$R" && export TMPDIR=/tmp
SW_RUNNER_TRACE=1 timeout -k 10 300 python -u bench.py --steps 60 --warmup 10 > "$O/bench_trace.log" 2>&1 || exit 1
tail -1 "$O/bench_trace.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1),"M/s", d["ms_per_step"], "ms", d["detail"]["runner_trace_ms_per_step"])'
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 "$R/bench.py" --steps 20 --warmup 3 > "$O/prof/log" 2>&1 && echo prof-ok
