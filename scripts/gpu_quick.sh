#!/bin/bash
# Quick GPU validation: GPU tests -> smoke -> headline bench (20 + 50 steps) -> H2D copy-engine probe
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/quick
cd "$R" && export TMPDIR=/tmp && mkdir -p $O
timeout -k 10 900 python -m pytest tests -m gpu -q > $O/pytest_gpu.log 2>&1 && echo "pytest gpu ok" && tail -1 $O/pytest_gpu.log &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log &&
timeout -k 10 400 python bench.py > $O/bench_default.log 2>&1 && tail -1 $O/bench_default.log | cut -c1-200 &&
timeout -k 10 400 python bench.py --steps 50 --warmup 10 > $O/bench_50.log 2>&1 && tail -1 $O/bench_50.log | cut -c1-200 &&
timeout -k 10 300 python scripts/probe_h2d.py > $O/probe_h2d.log 2>&1; cat $O/probe_h2d.log
