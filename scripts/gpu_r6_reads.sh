#!/bin/bash
# Round 6: reads while ingesting at every context cardinality: bench.py with 10,000
# customers and one asset per device (both above the trailer's per-key limit: routed through their
# assignments' page zone maps), >= 500 durable blocks, reader threads cycling through listings by
# assignment / area / customer / asset, by id and by alternate id (hit and miss).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r6_reads}
mkdir -p $O
STEPS=${STEPS:-700}
ARGS="--n-customers 10000 --n-assets 0"
timeout -k 10 400 python -u bench.py --steps $STEPS --warmup 5 $ARGS > $O/noreads.json 2> $O/noreads.err || exit $?
for R in ${READERS:-1 2}; do
  timeout -k 10 400 python -u bench.py --steps $STEPS --warmup 5 $ARGS --read-threads $R \
      > $O/reads${R}.json 2> $O/reads${R}.err || exit $?
done
