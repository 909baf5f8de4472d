#!/bin/bash
# Round 5: the headline bench (driver shape, index trailers in the step), then ingest with reader
# threads querying the store it writes (list by assignment / area, by id, by alternate id): back to
# back, and paced (a query every PACE ms per reader); and the same run length without readers.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
O=${1:-r5r}
STEPS=${STEPS:-1500}
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${O}_bench.json 2> gpurun_out/${O}_bench.err || exit $?
timeout -k 10 400 python -u bench.py --steps $STEPS --warmup 5 > gpurun_out/${O}_noreads.json 2> gpurun_out/${O}_noreads.err || exit $?
for R in ${READERS:-1 2}; do
  timeout -k 10 400 python -u bench.py --steps $STEPS --warmup 5 --read-threads $R \
      > gpurun_out/${O}_reads${R}.json 2> gpurun_out/${O}_reads${R}.err || exit $?
done
timeout -k 10 400 python -u bench.py --steps $STEPS --warmup 5 --read-threads 2 --read-pause-ms ${PACE:-20} \
    > gpurun_out/${O}_paced.json 2> gpurun_out/${O}_paced.err || exit $?
