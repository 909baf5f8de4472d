#!/bin/bash
# Round 6: the per-event path (reference deployment shape: infra server + service processes + N
# inbound-processing replicas in one consumer group) on the GPU box's host cores, 1 / 2 / 4 replicas.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r6_per_event_box}
mkdir -p $O
export TMPDIR=/tmp
for R in ${REPLICAS:-1 2 4}; do
  timeout -k 10 400 python -u scripts/bench_reference_config.py --path per-event --replicas $R \
      --events ${EVENTS:-40000} --paced 500 > $O/replicas$R.json 2> $O/replicas$R.err || exit $?
  tail -c 400 $O/replicas$R.json
done
