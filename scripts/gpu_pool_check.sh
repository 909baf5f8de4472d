#!/bin/bash
# Headline bench + 1M tenant path after sizing pinned row buffers to the step's rows.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/${1:-pool_check}
cd "$R" && mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench_default.log 2>&1 && tail -1 $O/bench_default.log | cut -c1-160 &&
run() {  # name args...
  n=$1; shift
  timeout -k 10 300 python scripts/bench_tenant_path.py --devices 20000 "$@" > $O/$n.log 2>&1 && tail -1 $O/$n.log | cut -c1-240
}
run copy_1m --batch 1048576 --batches 60 --max-msgs 1048576 --via-bus --store-retention 8388608 --no-zero-copy &&
run zc_1m --batch 1048576 --batches 60 --max-msgs 1048576 --via-bus --store-retention 8388608 --zero-copy &&
run copy_64k_bus --batch 65536 --batches 60 --max-msgs 65536 --via-bus --store-retention 524288 --no-zero-copy
