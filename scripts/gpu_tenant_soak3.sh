#!/bin/bash
# Soak at the other batch sizes: 200 x 1M and 1500 x 64K payloads through the raw topic, bounded
# 8-batch windows, zero-copy rows vs copied payloads.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/${1:-tenant_soak3}
cd "$R" && mkdir -p $O
run() {  # name args...
  n=$1; shift
  timeout -k 10 500 python -u scripts/bench_tenant_path.py --devices 20000 "$@" > $O/$n.log 2>&1 && tail -1 $O/$n.log | cut -c1-120
}
run zc_1m_200 --batch 1048576 --batches 200 --max-msgs 1048576 --via-bus --store-retention 8388608 --zero-copy &&
run copy_1m_200 --batch 1048576 --batches 200 --max-msgs 1048576 --via-bus --store-retention 8388608 --no-zero-copy &&
run zc_64k_1500 --batch 65536 --batches 1500 --max-msgs 65536 --via-bus --store-retention 524288 --zero-copy &&
run copy_64k_1500 --batch 65536 --batches 1500 --max-msgs 65536 --via-bus --store-retention 524288 --no-zero-copy
