#!/bin/bash
# Tenant path (whole instance, gpu-columnar) at large batches + the synchronous step breakdown.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/tenant_big
cd "$R" && mkdir -p $O
timeout -k 10 300 python scripts/probe_tenant_step.py --batch 262144 --batch 1048576 --iters 10 > $O/probe.log 2>&1 && tail -1 $O/probe.log &&
timeout -k 10 400 python scripts/bench_tenant_path.py --devices 20000 --batch 262144 --batches 40 > $O/t256k.log 2>&1 && tail -1 $O/t256k.log &&
timeout -k 10 400 python scripts/bench_tenant_path.py --devices 20000 --batch 1048576 --batches 20 --max-msgs 1048576 > $O/t1m.log 2>&1 && tail -1 $O/t1m.log
