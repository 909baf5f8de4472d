#!/bin/bash
# Final round-4 pass: GPU tests, smoke, bench + kernel profile, the 64K tenant path (with the host
# stack sampler on the first configuration)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > gpurun_out/fin_tests.log 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke.log 2>&1 || exit $?
bash scripts/gpu_bench_prof.sh fin || exit $?
bash scripts/gpu_tenant_sample.sh || exit $?
bash scripts/gpu_r4_tenant.sh r4_tenant_final
