#!/bin/bash
# Tenant path at small batches (64K payloads) with rows framed in place: direct and through the
# raw-payload topic, with the per-stage trace (SW_TENANT_TRACE) for the breakdown.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/${1:-tenant_small}
cd "$R" && mkdir -p $O
run() {  # name args...
  n=$1; shift
  SW_TENANT_TRACE=1 timeout -k 10 300 python scripts/bench_tenant_path.py --devices 20000 "$@" > $O/$n.log 2>&1 && tail -1 $O/$n.log | cut -c1-200
}
run direct_64k --batch 65536 --batches 60 &&
run bus_64k --batch 65536 --batches 60 --via-bus --max-msgs 65536 --store-retention 524288 &&
run bus_64k_copy --batch 65536 --batches 60 --via-bus --max-msgs 65536 --store-retention 524288 --no-zero-copy
