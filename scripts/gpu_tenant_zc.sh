#!/bin/bash
# Tenant path after the zero-copy changes: GPU tests, then whole-instance gpu-columnar throughput
# (direct process_batch calls, and through the raw-payload topic as event sources feed it).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/tenant_zc
cd "$R" && mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for b in 262144 1048576; do
  n=$(( b == 262144 ? 40 : 20 ))
  timeout -k 10 400 python scripts/bench_tenant_path.py --devices 20000 --batch $b --batches $n --max-msgs $b > $O/direct_$b.log 2>&1 && tail -1 $O/direct_$b.log || exit 1
  timeout -k 10 400 python scripts/bench_tenant_path.py --devices 20000 --batch $b --batches $n --max-msgs $b --via-bus > $O/bus_$b.log 2>&1 && tail -1 $O/bus_$b.log || exit 1
done
