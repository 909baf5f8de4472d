#!/bin/bash
# rocprofv3 kernel + memcopy trace of a short bench run; summaries land in gpurun_out/prof.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
mkdir -p "$R/gpurun_out/prof"
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" --steps ${STEPS:-10} --warmup ${WARM:-3} ${BENCH_ARGS} > "$R/gpurun_out/prof/bench_prof.log" 2>&1
rc=$?
find "$R/gpurun_out/prof" -name "*stats*.csv" | head -20
exit $rc
