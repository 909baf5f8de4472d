#!/bin/bash
# Round-4 GPU pass: tests + bench profile, copy-engine variants, N>1 rehearsal (gloo, shared GPU),
# then the 64K tenant path.  Each step has its own time limit; the first failure ends the pass.
set -o pipefail
cd "$(dirname "$0")/.."
T=${1:-fold2}
bash scripts/gpu_fold.sh $T && \
bash scripts/gpu_sdma_var.sh sdma && \
NS="2 4" bash scripts/gpu_rehearse_multirank.sh && \
bash scripts/gpu_r4_tenant.sh r4_tenant
