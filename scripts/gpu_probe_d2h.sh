#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && export TMPDIR=/tmp && mkdir -p gpurun_out/d2h
true &&
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/d2h/prof" -o run -- python3 "$R/scripts/probe_d2h.py" > "$R/gpurun_out/d2h/prof.log" 2>&1 && echo "prof ok"
