#!/bin/bash
# ~1B-event durable store on one MI355X: bench.py ingests (blocks kept), then the read benchmark
# indexes and queries them.  Steps are sized to the free space of the scratch disk (~40 B / event
# with indexes).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
D=${SW_STORE_DIR:-/tmp/sw-store-reads}
rm -rf "$D"; mkdir -p "$D"
df -B1 "$D" > gpurun_out/store_df.txt
STEPS=$(python3 -c "
import shutil; free = shutil.disk_usage('$D').free
print(max(20, min(${STEPS:-1000}, int(free * 0.7 / (40 * 1.05e6)))))")
echo "steps $STEPS" > gpurun_out/store_steps.txt
timeout -k 10 900 python -u bench.py --steps "$STEPS" --warmup 5 --durable-dir "$D" --durable-retention-gb 0 \
    > gpurun_out/store_ingest.json 2> gpurun_out/store_ingest.err || { tail -5 gpurun_out/store_ingest.err; rm -rf "$D"; exit 1; }
timeout -k 10 1200 python -u scripts/bench_store_reads.py --dir "$D/rank0" --queries 100 \
    > gpurun_out/store_reads.json 2> gpurun_out/store_reads.err
rc=$?
rm -rf "$D"
exit $rc
