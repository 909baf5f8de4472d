#!/bin/bash
# GPU tests, the driver's bench shape (20 steps / 5 warmup) x3, the default bench, a runner trace and
# a kernel profile.  Results under gpurun_out/<name>.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${1:-r3_final}"
mkdir -p "$O/prof" && cd "$R" && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/b20_$i.log" 2>&1 || exit 1
  tail -1 "$O/b20_$i.log" | cut -c1-170
done
timeout -k 10 300 python -u bench.py > "$O/bench_default.log" 2>&1 || exit 1
tail -1 "$O/bench_default.log" | cut -c1-170
SW_RUNNER_TRACE=1 timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 > "$O/bench_trace.log" 2>&1 || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 "$R/bench.py" --steps 20 --warmup 3 > "$O/prof/log" 2>&1 && echo prof-ok
