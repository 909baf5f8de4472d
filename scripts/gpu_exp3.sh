#!/bin/bash
# outbound-mode comparison: direct (zero-copy stores) vs sdma (HBM staging + async D2H) vs push
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && export TMPDIR=/tmp && mkdir -p gpurun_out/exp3
run() { name=$1; shift; timeout -k 10 300 env "$@" > gpurun_out/exp3/$name.log 2>&1; rc=$?; echo "$name rc=$rc $(tail -1 gpurun_out/exp3/$name.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"]/1e6, "M ev/s", d["ms_per_step"], "ms")' 2>/dev/null)"; return $rc; }
timeout -k 10 600 python -m pytest tests/test_gpu_engine.py tests/test_services.py -m gpu -x -q > gpurun_out/exp3/pytest_gpu.log 2>&1 && echo "pytest gpu ok" &&
run sdma SW_OUTBOUND_MODE=sdma python bench.py --steps 20 --warmup 5 &&
run direct SW_OUTBOUND_MODE=direct python bench.py --steps 20 --warmup 5 &&
run sdma2m SW_OUTBOUND_MODE=sdma python bench.py --steps 10 --warmup 3 --msgs 2097152 &&
cd /tmp && timeout -k 10 300 env SW_OUTBOUND_MODE=sdma rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/exp3/prof" -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 > "$R/gpurun_out/exp3/prof.log" 2>&1 && echo "prof ok"
