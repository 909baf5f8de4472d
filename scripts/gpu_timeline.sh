#!/bin/bash
# Kernel + memory-copy timeline of a short durable bench (overlap of H2D, compute and D2H).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${1:-timeline}"
mkdir -p "$O" && cd /tmp && export TMPDIR=/tmp
SW_PIPELINE_DEPTH=${DEPTH:-2} SW_ROUTE_THREADS=${RT:-4} timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$O" -o run -- python3 "$R/bench.py" --steps 30 --warmup 5 > "$O/log" 2>&1 && echo timeline-ok
