#!/bin/bash
# A/B of the XCD-aware block-id remap: GPU tests, bench and rocprofv3 kernel stats with each library.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/xcd
X="$R/sitewhere_amd/_lib/libswgpu_xcd.so"
cd "$R" && export TMPDIR=/tmp && mkdir -p $O/prof_default $O/prof_xcd
SW_GPU_LIB="$X" timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_xcd.log 2>&1 && echo "pytest gpu (xcd lib) ok" && tail -1 $O/pytest_xcd.log &&
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > $O/bench_default_a.log 2>&1 && tail -1 $O/bench_default_a.log | cut -c1-120 &&
SW_GPU_LIB="$X" timeout -k 10 300 python bench.py --steps 50 --warmup 10 > $O/bench_xcd_a.log 2>&1 && tail -1 $O/bench_xcd_a.log | cut -c1-120 &&
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > $O/bench_default_b.log 2>&1 && tail -1 $O/bench_default_b.log | cut -c1-120 &&
SW_GPU_LIB="$X" timeout -k 10 300 python bench.py --steps 50 --warmup 10 > $O/bench_xcd_b.log 2>&1 && tail -1 $O/bench_xcd_b.log | cut -c1-120 &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_default" -o run -- python3 "$R/bench.py" --steps 20 --warmup 3 > "$R/$O/prof_default/log" 2>&1 && echo "prof default ok" &&
export SW_GPU_LIB="$X" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_xcd" -o run -- python3 "$R/bench.py" --steps 20 --warmup 3 > "$R/$O/prof_xcd/log" 2>&1 && echo "prof xcd ok"
