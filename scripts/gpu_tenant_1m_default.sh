#!/bin/bash
# 1M-payload batches with the store's default window (every batch kept): zero-copy rows (pool
# fills, then spill buffers) vs copied payloads; and through the topic with bounded windows.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/${1:-tenant_1m_default}
cd "$R" && mkdir -p $O
run() {  # name args...
  n=$1; shift
  timeout -k 10 300 python scripts/bench_tenant_path.py --devices 20000 "$@" > $O/$n.log 2>&1 && tail -1 $O/$n.log | cut -c1-120
}
run zc_1m_direct --batch 1048576 --batches 60 --max-msgs 1048576 --zero-copy &&
run copy_1m_direct --batch 1048576 --batches 60 --max-msgs 1048576 --no-zero-copy &&
run zc_256k_bus --batch 262144 --batches 100 --max-msgs 262144 --via-bus --store-retention 2097152 --zero-copy &&
run copy_256k_bus --batch 262144 --batches 100 --max-msgs 262144 --via-bus --store-retention 2097152 --no-zero-copy
