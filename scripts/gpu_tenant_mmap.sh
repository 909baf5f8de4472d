#!/bin/bash
# Copied columnar payloads land in fresh malloc memory each batch.  Large blocks are mmap'ed by
# glibc and page-faulted on first touch; with a high mmap threshold they are reused from the heap.
# A/B on the tenant path through the topic (copied payloads, bounded windows).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/${1:-tenant_mmap}
cd "$R" && mkdir -p $O
run() {  # name env args...
  n=$1; e=$2; shift 2
  env $e timeout -k 10 300 python scripts/bench_tenant_path.py --devices 20000 "$@" > $O/$n.log 2>&1 && tail -1 $O/$n.log | cut -c1-120
}
HI="MALLOC_MMAP_THRESHOLD_=1073741824 MALLOC_TRIM_THRESHOLD_=8589934592"
run base_1m "X=1" --batch 1048576 --batches 60 --max-msgs 1048576 --via-bus --store-retention 8388608 &&
run heap_1m "$HI" --batch 1048576 --batches 60 --max-msgs 1048576 --via-bus --store-retention 8388608 &&
run base_64k "X=1" --batch 65536 --batches 60 --max-msgs 65536 --via-bus --store-retention 524288 &&
run heap_64k "$HI" --batch 65536 --batches 60 --max-msgs 65536 --via-bus --store-retention 524288 &&
run base_64k_direct "X=1" --batch 65536 --batches 60 &&
run heap_64k_direct "$HI" --batch 65536 --batches 60
