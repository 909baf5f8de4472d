#!/bin/bash
# gpu tests -> bench -> rocprofv3 kernel trace (no memory-copy trace: it segfaults at exit on this image)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && export TMPDIR=/tmp && mkdir -p gpurun_out/prof
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest gpu ok" &&
timeout -k 10 400 python bench.py --steps ${STEPS:-20} --warmup ${WARM:-5} ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 && echo "bench ok" && tail -1 gpurun_out/bench.log &&
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 ${BENCH_ARGS} > "$R/gpurun_out/prof/log" 2>&1 && echo "prof ok"
