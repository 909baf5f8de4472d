#!/bin/bash
# Quick GPU check after a kernel change: GPU tests -> 50-step bench -> rocprofv3 kernel stats.
#   bash scripts/gpu_quick.sh <name>     (results under gpurun_out/<name>)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/${1:-quick}
cd "$R" && export TMPDIR=/tmp && mkdir -p $O/prof
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && echo "pytest gpu ok" && tail -1 $O/pytest_gpu.log &&
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > $O/bench_50.log 2>&1 && tail -1 $O/bench_50.log | cut -c1-140 &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof" -o run -- python3 "$R/bench.py" --steps 20 --warmup 3 > "$R/$O/prof/log" 2>&1 && echo "prof ok"
