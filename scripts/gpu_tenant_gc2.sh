#!/bin/bash
# GC A/B on the tenant path at 1M-payload batches: no tuning (SW_GC_TUNE=0), the tenant's own
# tuning at start (freeze + thresholds), and a second freeze after the devices are loaded.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/${1:-tenant_gc2}
cd "$R" && mkdir -p $O
run() {  # name batch batches env gc
  env $4 SW_TENANT_TRACE=1 timeout -k 10 400 python scripts/bench_tenant_path.py --devices 20000 --batch $2 --batches $3 --max-msgs $2 --via-bus --store-retention $(( 8 * $2 )) --gc $5 > $O/$1.log 2>&1 && tail -1 $O/$1.log | cut -c1-160
}
run off_1m 1048576 60 SW_GC_TUNE=0 default &&
run tenant_1m 1048576 60 SW_GC_TUNE=1 default &&
run both_1m 1048576 60 SW_GC_TUNE=1 freeze &&
run off_1m_b 1048576 60 SW_GC_TUNE=0 default &&
run tenant_256k 262144 120 SW_GC_TUNE=1 default
