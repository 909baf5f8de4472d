#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && export TMPDIR=/tmp && mkdir -p gpurun_out/exp
run() { name=$1; shift; timeout -k 10 300 env "$@" > gpurun_out/exp/$name.log 2>&1; rc=$?; echo "$name rc=$rc $(tail -1 gpurun_out/exp/$name.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"]/1e6, "M ev/s", d["ms_per_step"], "ms")' 2>/dev/null)"; return $rc; }
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest gpu ok" &&
run push SW_OUTBOUND_MODE=push python bench.py --steps 20 --warmup 5 &&
run direct SW_OUTBOUND_MODE=direct python bench.py --steps 20 --warmup 5 &&
run no_outbound python bench.py --steps 20 --warmup 5 --no-outbound &&
run push2m SW_OUTBOUND_MODE=push python bench.py --steps 10 --warmup 3 --msgs 2097152
