#!/bin/bash
# One GPU-box round: gpu tests -> smoke -> short bench.  Each GPU step has its own time limit;
# steps are chained with && so a fault/timeout ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=${STEPS:-10}
WARM=${WARM:-3}
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest gpu ok" &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 400 python bench.py --steps $STEPS --warmup $WARM > gpurun_out/bench.log 2>&1 && echo "bench ok" && tail -1 gpurun_out/bench.log
