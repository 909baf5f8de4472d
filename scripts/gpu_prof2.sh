#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
mkdir -p "$R/gpurun_out/probe" "$R/gpurun_out/prof2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/probe" -o run -- python3 "$R/scripts/prof_probe.py" > "$R/gpurun_out/probe/log" 2>&1 && echo "probe ok" &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof2" -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 > "$R/gpurun_out/prof2/log" 2>&1 && echo "bench prof ok"
rc=$?
find "$R/gpurun_out/probe" "$R/gpurun_out/prof2" -name "*.csv" | head
exit $rc
