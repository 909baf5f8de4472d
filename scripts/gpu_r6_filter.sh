#!/bin/bash
# Round 6: generational dedup filter on the MI355X -- its GPU tests (oracle / native parity, rotation
# past retention at bench scale, multi-rank settling), the smoke step, then the bench.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r6_filter}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_dedup_window.py \
    tests/test_gpu_bench_scale.py tests/test_multirank_strings.py -m gpu > $O/tests.log 2>&1 || exit $?
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), "M/s", d["ms_per_step"], d["detail"]["durable"]["bytes_per_event"], d["detail"]["rejected_rank0"])'
