#!/bin/bash
# Service-level MI355X path at three batch sizes (gpu-columnar tenant of a whole instance).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/tenant
cd "$R" && export TMPDIR=/tmp && mkdir -p $O
timeout -k 10 400 python scripts/bench_tenant_path.py --devices 20000 --batch 65536 --batches 30 > $O/b64k.log 2>&1 && tail -1 $O/b64k.log &&
timeout -k 10 400 python scripts/bench_tenant_path.py --devices 20000 --batch 262144 --batches 20 --max-msgs 262144 > $O/b256k.log 2>&1 && tail -1 $O/b256k.log &&
timeout -k 10 400 python scripts/bench_tenant_path.py --devices 20000 --batch 1048576 --batches 10 --max-msgs 1048576 > $O/b1m.log 2>&1 && tail -1 $O/b1m.log
