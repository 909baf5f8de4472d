#!/bin/bash
# Full GPU validation: GPU tests -> smoke -> headline bench -> tenant-path bench -> rocprofv3 kernel stats
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/${1:-full}
cd "$R" && export TMPDIR=/tmp && mkdir -p $O/prof
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && echo "pytest gpu ok" && tail -1 $O/pytest_gpu.log &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log &&
timeout -k 10 400 python bench.py > $O/bench_default.log 2>&1 && tail -1 $O/bench_default.log | cut -c1-160 &&
timeout -k 10 400 python bench.py --steps 50 --warmup 10 > $O/bench_50.log 2>&1 && tail -1 $O/bench_50.log | cut -c1-160 &&
timeout -k 10 600 python scripts/bench_tenant_path.py --devices 20000 --batch 65536 --batches 30 > $O/bench_tenant.log 2>&1 && tail -1 $O/bench_tenant.log &&
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof" -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 > "$R/$O/prof/log" 2>&1 && echo "prof ok" &&
cd "$R" && python scripts/summarize_prof.py "$O/prof/run_kernel_trace.csv" > "$O/top_kernels.md"
