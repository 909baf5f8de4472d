#!/bin/bash
# explicit SDMA (HSA copy engine) outbound vs direct stores
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && export TMPDIR=/tmp && mkdir -p gpurun_out/exp5
run() { name=$1; shift; timeout -k 10 200 env "$@" > gpurun_out/exp5/$name.log 2>&1; rc=$?; echo "$name rc=$rc $(tail -1 gpurun_out/exp5/$name.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"]/1e6, "M ev/s", d["ms_per_step"], "ms")' 2>/dev/null)"; return $rc; }
B="python bench.py --steps 20 --warmup 5"
timeout -k 10 300 python -m pytest tests/test_gpu_engine.py -x -q > gpurun_out/exp5/pytest.log 2>&1 && echo "pytest ok" &&
run hsa0 SW_OUTBOUND_MODE=hsa $B &&
run hsa1 SW_OUTBOUND_MODE=hsa SW_SDMA_ENGINE=1 $B &&
run hsa2 SW_OUTBOUND_MODE=hsa SW_SDMA_ENGINE=2 $B &&
run direct SW_OUTBOUND_MODE=direct $B &&
cd /tmp && timeout -k 10 300 env SW_OUTBOUND_MODE=hsa rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/exp5/prof" -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 > "$R/gpurun_out/exp5/prof.log" 2>&1 && echo "prof ok"
