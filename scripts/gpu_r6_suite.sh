#!/bin/bash
# Round 6: the GPU test suite and smoke() on one box, as the driver runs them at round end.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r6_suite}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
RC=$?
tail -5 $O/pytest_gpu.log
[ $RC -eq 0 ] || exit $RC
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
