#!/bin/bash
# pipeline depth with copy-engine outbound
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && export TMPDIR=/tmp && mkdir -p gpurun_out/exp6
run() { name=$1; shift; timeout -k 10 200 env "$@" > gpurun_out/exp6/$name.log 2>&1; rc=$?; echo "$name rc=$rc $(tail -1 gpurun_out/exp6/$name.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"]/1e6, "M ev/s", d["ms_per_step"], "ms")' 2>/dev/null)"; return $rc; }
B="python bench.py --steps 30 --warmup 5"
timeout -k 10 300 python -m pytest tests/test_gpu_engine.py -x -q > gpurun_out/exp6/pytest.log 2>&1 && echo "pytest ok" &&
run hsa_b2 SW_PIPELINE_BUFFERS=2 $B &&
run hsa_b3 SW_PIPELINE_BUFFERS=3 $B &&
run hsa_b3_e2 SW_PIPELINE_BUFFERS=3 SW_SDMA_ENGINE=2 $B &&
run hsa_b3_e3 SW_PIPELINE_BUFFERS=3 SW_SDMA_ENGINE=3 $B &&
run hsa_b3_2m SW_PIPELINE_BUFFERS=3 python bench.py --steps 15 --warmup 3 --msgs 2097152 &&
run hsa_b3_512k SW_PIPELINE_BUFFERS=3 python bench.py --steps 40 --warmup 5 --msgs 524288
