#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && export TMPDIR=/tmp && mkdir -p gpurun_out/tenant
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/tenant/pytest_gpu.log 2>&1 && echo "pytest gpu ok" && tail -1 gpurun_out/tenant/pytest_gpu.log &&
timeout -k 10 600 python scripts/bench_tenant_path.py --devices 20000 --batch 65536 --batches 30 > gpurun_out/tenant/bench_tenant.log 2>&1 && tail -1 gpurun_out/tenant/bench_tenant.log
