#!/bin/bash
# Round 5: index-trailer GPU tests, the heads probe, then the bench (driver shape) + its kernel profile
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
O=${1:-r5}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_index.py tests/test_gpu_segments.py > gpurun_out/${O}_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/ix_probe.py > gpurun_out/${O}_probe.json 2> gpurun_out/${O}_probe.err || exit $?
bash scripts/gpu_bench_prof.sh ${O} || exit $?
python scripts/step_dispatches.py gpurun_out/${O}_prof/run_results.db --step 12 > gpurun_out/${O}_dispatches.md 2>&1 || true
