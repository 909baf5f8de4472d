#!/bin/bash
# Tenant path at 1M-payload batches with and without MALLOC_ARENA_MAX=1 (the store thread's
# multi-MB columnar payloads come from a per-thread malloc arena whose heaps are unmapped and
# re-faulted batch after batch; one arena reuses the main heap).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/${1:-tenant_arena}
cd "$R" && mkdir -p $O
for b in 262144 1048576; do
  n=$(( b == 262144 ? 120 : 60 ))
  SW_TENANT_TRACE=1 timeout -k 10 400 python scripts/bench_tenant_path.py --devices 20000 --batch $b --batches $n --max-msgs $b --via-bus --store-retention $(( 8 * b )) > $O/default_$b.log 2>&1 && tail -1 $O/default_$b.log | cut -c1-400 || exit 1
  MALLOC_ARENA_MAX=1 SW_TENANT_TRACE=1 timeout -k 10 400 python scripts/bench_tenant_path.py --devices 20000 --batch $b --batches $n --max-msgs $b --via-bus --store-retention $(( 8 * b )) > $O/arena1_$b.log 2>&1 && tail -1 $O/arena1_$b.log | cut -c1-400 || exit 1
done
