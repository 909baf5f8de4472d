#!/bin/bash
# Round-3 durable path on the MI355X: encoder + engine GPU tests, then the durable bench and the
# same bench without the durable store (attribution).  Results under gpurun_out/<name>.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${1:-r3_durable}"
mkdir -p "$O" && cd "$R" && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_segments.py tests/test_gpu_engine.py -x -v --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1; rc=$?
tail -3 "$O/pytest.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 > "$O/bench_durable.log" 2>&1 && tail -1 "$O/bench_durable.log" | cut -c1-400 &&
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --no-durable > "$O/bench_nodurable.log" 2>&1 && tail -1 "$O/bench_nodurable.log" | cut -c1-300
