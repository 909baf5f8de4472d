#!/bin/bash
# Bus-through engine: GPU tests, then the headline bench with and without the commit-log hop.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/bus
cd "$R" && mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_bus.py tests/test_gpu_engine.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-bus > $O/bench_nobus.log 2>&1 && tail -1 $O/bench_nobus.log | cut -c1-200 &&
timeout -k 10 300 python bench.py > $O/bench_bus.log 2>&1 && tail -1 $O/bench_bus.log | cut -c1-200 &&
timeout -k 10 300 python bench.py --no-bus > $O/bench_nobus2.log 2>&1 && tail -1 $O/bench_nobus2.log | cut -c1-200 &&
timeout -k 10 300 python bench.py > $O/bench_bus2.log 2>&1 && tail -1 $O/bench_bus2.log | cut -c1-200
