#!/bin/bash
# Round 6: bench (driver shape) + its rocprofv3 kernel trace, summarised on the box (per-kernel
# steady-state totals + one step's dispatch sequence); the trace database is deleted afterwards.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${1:-r6_kernels}"
P="$R/gpurun_out/${1:-r6_kernels}_db"
mkdir -p "$O" && cd "$R" && export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > "$O/bench.json" 2> "$O/bench.err" || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$P" -o run -- \
    python -u "$R/bench.py" --steps 20 --warmup 5 ${BENCH_ARGS:-} > "$O/prof_bench.json" 2> "$O/prof.err" || exit $?
cd "$R"
DB=$(ls "$P"/*.db "$P"/*/*.db 2>/dev/null | head -1)
python scripts/step_dispatches.py "$DB" --step 8 --stats > "$O/kernel_stats.md" 2>&1
python scripts/step_dispatches.py "$DB" --step 12 > "$O/step_dispatches.md" 2>&1
rm -rf "$P"
cat "$O/bench.json"; tail -3 "$O/kernel_stats.md"
