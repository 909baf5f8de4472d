#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && export TMPDIR=/tmp && mkdir -p gpurun_out/d2h
timeout -k 10 120 python scripts/probe_d2h.py > gpurun_out/d2h/plain.log 2>&1 && cat gpurun_out/d2h/plain.log &&
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/d2h/prof" -o run -- python3 "$R/scripts/probe_d2h.py" > "$R/gpurun_out/d2h/prof.log" 2>&1 && echo "prof ok"
