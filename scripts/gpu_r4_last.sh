#!/bin/bash
# Last round-4 pass on the final tree: GPU tests, smoke, bench + kernel profile, then the 64K
# tenant path with and without alternate ids (store-backed dedup lookups in one native pass)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > gpurun_out/last_tests.log 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/last_smoke.log 2>&1 || exit $?
bash scripts/gpu_bench_prof.sh last || exit $?
bash scripts/gpu_tenant_alt.sh last_tenant_alt
