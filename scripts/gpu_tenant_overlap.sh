#!/bin/bash
# Overlapped tenant steps: GPU tests, then whole-instance gpu-columnar throughput through the
# raw-payload topic (zero-copy pinned records, as event sources feed it) at 256K and 1M batches.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/${1:-tenant_overlap}
cd "$R" && mkdir -p $O
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for b in 262144 1048576; do
  n=$(( b == 262144 ? 40 : 20 ))
  SW_TENANT_TRACE=1 timeout -k 10 400 python scripts/bench_tenant_path.py --devices 20000 --batch $b --batches $n --max-msgs $b --via-bus > $O/bus_$b.log 2>&1 && tail -1 $O/bus_$b.log || exit 1
  SW_TENANT_TRACE=1 timeout -k 10 400 python scripts/bench_tenant_path.py --devices 20000 --batch $b --batches $(( n * 3 )) --max-msgs $b --via-bus --store-retention $(( 8 * b )) > $O/bus_ret_$b.log 2>&1 && tail -1 $O/bus_ret_$b.log || exit 1
done
