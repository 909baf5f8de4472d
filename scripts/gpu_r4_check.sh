#!/bin/bash
# Round-4 GPU check: lossless-record kernels (decode string refs, v2 block encoder) + a short bench
# and a kernel-stats profile.  Every GPU step has its own time limit; the chain stops at the first
# failure.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
    tests/test_gpu_decode.py tests/test_gpu_segments.py > gpurun_out/r4_gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4_bench.json 2> gpurun_out/r4_bench.err || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OLDPWD/gpurun_out/r4_prof" -o run -- \
    python -u "$OLDPWD/bench.py" --steps 20 --warmup 5 > "$OLDPWD/gpurun_out/r4_prof_bench.json" 2> "$OLDPWD/gpurun_out/r4_prof.err"
