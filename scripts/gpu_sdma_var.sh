#!/bin/bash
# bench variants: which copy engine the outbound / block D2H copies use (SW_SDMA_ENGINE, 0 = runtime)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
T=${1:-sdma}
for E in 1 2 3; do
  SW_SDMA_ENGINE=$E timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_e$E.json 2> gpurun_out/${T}_e$E.err || exit $?
done
