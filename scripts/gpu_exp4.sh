#!/bin/bash
# outbound off the critical path: few-WG push kernel / WG-limited blit vs direct stores
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && export TMPDIR=/tmp && mkdir -p gpurun_out/exp4
run() { name=$1; shift; timeout -k 10 200 env "$@" > gpurun_out/exp4/$name.log 2>&1; rc=$?; echo "$name rc=$rc $(tail -1 gpurun_out/exp4/$name.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"]/1e6, "M ev/s", d["ms_per_step"], "ms")' 2>/dev/null)"; return $rc; }
B="python bench.py --steps 20 --warmup 5"
run direct SW_OUTBOUND_MODE=direct $B &&
run push8 SW_OUTBOUND_MODE=push SW_PUSH_BLOCKS=8 $B &&
run push16 SW_OUTBOUND_MODE=push SW_PUSH_BLOCKS=16 $B &&
run push32 SW_OUTBOUND_MODE=push SW_PUSH_BLOCKS=32 $B &&
run push64 SW_OUTBOUND_MODE=push SW_PUSH_BLOCKS=64 $B &&
run sdma_wg8 SW_OUTBOUND_MODE=sdma DEBUG_CLR_LIMIT_BLIT_WG=8 $B &&
run sdma_wg16 SW_OUTBOUND_MODE=sdma DEBUG_CLR_LIMIT_BLIT_WG=16 $B &&
run sdma_wg32 SW_OUTBOUND_MODE=sdma DEBUG_CLR_LIMIT_BLIT_WG=32 $B &&
run noout python bench.py --steps 20 --warmup 5 --no-outbound
