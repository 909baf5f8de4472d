#!/bin/bash
# full GPU test suite -> smoke -> bench (default config) -> rocprofv3 kernel stats
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && export TMPDIR=/tmp && mkdir -p gpurun_out/r3/prof
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/r3/pytest_gpu.log 2>&1 && echo "pytest gpu ok" && tail -2 gpurun_out/r3/pytest_gpu.log &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3/smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 400 python bench.py > gpurun_out/r3/bench_default.log 2>&1 && echo "bench ok" && tail -1 gpurun_out/r3/bench_default.log &&
timeout -k 10 400 python bench.py --steps 50 --warmup 10 > gpurun_out/r3/bench_50.log 2>&1 && tail -1 gpurun_out/r3/bench_50.log &&
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r3/prof" -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 > "$R/gpurun_out/r3/prof/log" 2>&1 && echo "prof ok"
