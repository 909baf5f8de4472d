#!/bin/bash
# GPU tests (all) then the durable headline bench.  Results under gpurun_out/<name>.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${1:-r3_check}"
mkdir -p "$O" && cd "$R" && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1; rc=$?
tail -3 "$O/pytest.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps ${STEPS:-100} --warmup 10 > "$O/bench.log" 2>&1; rc=$?
tail -1 "$O/bench.log" | cut -c1-4000
exit $rc
