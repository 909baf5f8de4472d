#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && export TMPDIR=/tmp && mkdir -p gpurun_out/exp
run() { name=$1; shift; timeout -k 10 300 env "$@" > gpurun_out/exp/$name.log 2>&1; rc=$?; echo "$name rc=$rc $(tail -1 gpurun_out/exp/$name.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"]/1e6, "M ev/s", d["ms_per_step"], "ms")' 2>/dev/null)"; return $rc; }
run default python bench.py --steps 20 --warmup 5 &&
run sdma1 HSA_ENABLE_SDMA=1 python bench.py --steps 20 --warmup 5 &&
run no_outbound python bench.py --steps 20 --warmup 5 --no-outbound &&
run sdma0 HSA_ENABLE_SDMA=0 python bench.py --steps 20 --warmup 5 &&
run half_msgs python bench.py --steps 20 --warmup 5 --msgs 524288 &&
run big_msgs python bench.py --steps 10 --warmup 3 --msgs 4194304
