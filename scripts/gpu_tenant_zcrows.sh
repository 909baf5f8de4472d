#!/bin/bash
# Zero-copy columnar payloads (header framed in front of the rows in the engine's pinned row
# buffers) vs the copied encoding, whole-instance tenant path through the raw-payload topic.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/${1:-tenant_zcrows}
cd "$R" && mkdir -p $O
[ -n "$SKIP_TESTS" ] || { timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc; }
run() {  # name batch batches flag
  SW_TENANT_TRACE=1 timeout -k 10 400 python scripts/bench_tenant_path.py --devices 20000 --batch $2 --batches $3 --max-msgs $2 --via-bus --store-retention $(( 8 * $2 )) $4 > $O/$1.log 2>&1 && tail -1 $O/$1.log | cut -c1-170
}
run zc_1m 1048576 60 --zero-copy && run copy_1m 1048576 60 --no-zero-copy &&
run zc_256k 262144 120 --zero-copy && run copy_256k 262144 120 --no-zero-copy &&
run zc_1m_b 1048576 60 --zero-copy
