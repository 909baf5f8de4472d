#!/bin/bash
# Tenant-path tail latency: default GC vs a frozen start-up heap (gc.freeze + higher gen-0
# threshold), 256K and 1M batches through the raw-payload topic with store retention.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/${1:-tenant_gc}
cd "$R" && mkdir -p $O
for b in 262144 1048576; do
  n=$(( b == 262144 ? 120 : 60 ))
  for g in default freeze; do
    SW_TENANT_TRACE=1 timeout -k 10 400 python scripts/bench_tenant_path.py --devices 20000 --batch $b --batches $n --max-msgs $b --via-bus --store-retention $(( 8 * b )) --gc $g > $O/${g}_$b.log 2>&1 && tail -1 $O/${g}_$b.log | cut -c1-200 || exit 1
  done
done
