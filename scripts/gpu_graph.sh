#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && export TMPDIR=/tmp && mkdir -p gpurun_out/graph
run() { name=$1; shift; timeout -k 10 200 env "$@" > gpurun_out/graph/$name.log 2>&1; rc=$?; echo "$name rc=$rc $(tail -1 gpurun_out/graph/$name.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"]/1e6, "M ev/s", d["ms_per_step"], "ms")' 2>/dev/null)"; return $rc; }
run g1_1m SW_GRAPH=1 python bench.py --steps 50 --warmup 10 &&
run g0_1m SW_GRAPH=0 python bench.py --steps 50 --warmup 10 &&
run g1_64k SW_GRAPH=1 python bench.py --steps 200 --warmup 20 --msgs 65536 &&
run g0_64k SW_GRAPH=0 python bench.py --steps 200 --warmup 20 --msgs 65536 &&
run g1_16k SW_GRAPH=1 python bench.py --steps 400 --warmup 20 --msgs 16384 &&
run g0_16k SW_GRAPH=0 python bench.py --steps 400 --warmup 20 --msgs 16384
