#!/bin/bash
# dispatch folding + string exchange: every GPU test, then bench + kernel profile
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
T=${1:-fold}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_multirank_strings.py \
    tests/test_multirank.py > gpurun_out/${T}_mr.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > gpurun_out/${T}_tests.log 2>&1 || exit $?
bash scripts/gpu_bench_prof.sh $T || exit $?
