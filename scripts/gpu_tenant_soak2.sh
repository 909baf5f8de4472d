#!/bin/bash
# Soak: 600 batches of 256K payloads through the raw topic, zero-copy rows, bounded windows; then
# the same copied.  Checks pool recycling over a long run (pinned_rows) and steady throughput.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/${1:-tenant_soak2}
cd "$R" && mkdir -p $O
run() {  # name args...
  n=$1; shift
  timeout -k 10 500 python -u scripts/bench_tenant_path.py --devices 20000 "$@" > $O/$n.log 2>&1 && tail -1 $O/$n.log | cut -c1-120
}
run zc_256k_600 --batch 262144 --batches 600 --max-msgs 262144 --via-bus --store-retention 2097152 --zero-copy &&
run copy_256k_600 --batch 262144 --batches 600 --max-msgs 262144 --via-bus --store-retention 2097152 --no-zero-copy
