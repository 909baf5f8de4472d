#!/bin/bash
# bench (driver shape) + a kernel-stats profile of the same run
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
O=${1:-bp}
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/${O}_bench.json 2> gpurun_out/${O}_bench.err || exit $?
R=$PWD
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${O}_prof" -o run -- \
    python -u "$R/bench.py" --steps 20 --warmup 5 ${BENCH_ARGS:-} > "$R/gpurun_out/${O}_prof_bench.json" 2> "$R/gpurun_out/${O}_prof.err"
