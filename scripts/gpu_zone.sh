#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && export TMPDIR=/tmp && mkdir -p gpurun_out/zone/prof
timeout -k 10 600 python -m pytest tests/test_gpu_engine.py tests/test_multirank.py -m gpu -x -q > gpurun_out/zone/pytest.log 2>&1 && echo "pytest ok" &&
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > gpurun_out/zone/bench.log 2>&1 && tail -1 gpurun_out/zone/bench.log | cut -c1-200 &&
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/zone/prof" -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 > "$R/gpurun_out/zone/prof/log" 2>&1 && echo "prof ok"
