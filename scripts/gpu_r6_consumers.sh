#!/bin/bash
# Round 6: the enriched-event consumers on the GPU box next to a live engine: bench.py
# ingests (durable, 1M payloads / step) in the background while scripts/bench_consumers.py runs the
# MQTT connector (area + event-type filters, event-type only) against a broker in its own process and
# the threshold rule (rare and frequent bounds), each over durable engine blocks.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r6_consumers}
mkdir -p $O
timeout -k 10 300 python -u scripts/bench_consumers.py --seconds ${SECONDS_PER:-10} --threads ${THREADS:-8} \
    > $O/consumers_alone.json 2> $O/consumers_alone.err || exit $?
timeout -k 10 600 python -u bench.py --steps ${STEPS:-30000} --warmup 5 > $O/bench_live.json 2> $O/bench_live.err &
BP=$!
sleep ${DELAY:-40}
timeout -k 10 300 python -u scripts/bench_consumers.py --seconds ${SECONDS_PER:-10} --threads ${THREADS:-8} \
    > $O/consumers_live.json 2> $O/consumers_live.err
RC=$?
wait $BP
BRC=$?
echo "consumers rc=$RC bench rc=$BRC"
cat $O/consumers_alone.json $O/consumers_live.json
exit $RC
