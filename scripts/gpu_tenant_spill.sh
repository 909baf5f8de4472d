#!/bin/bash
# zeroCopyRows with the store's default window (every batch kept): once the pinned row pool is
# held downstream, steps fall back to copying through spill buffers instead of allocating.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/${1:-tenant_spill}
cd "$R" && mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
run() {  # name args...
  n=$1; shift
  timeout -k 10 300 python scripts/bench_tenant_path.py --devices 20000 "$@" > $O/$n.log 2>&1 && tail -1 $O/$n.log | cut -c1-240
}
run direct_64k_zc --batch 65536 --batches 60 --zero-copy &&
run direct_64k_copy --batch 65536 --batches 60 --no-zero-copy
