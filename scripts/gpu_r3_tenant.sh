#!/bin/bash
# GPU tests, then the durable tenant path (gpu-columnar) at 256K and 1M-payload batches with 0% and
# 1% rejected payloads (unregistered devices).  Results under gpurun_out/<name>.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${1:-r3_tenant}"
mkdir -p "$O" && cd "$R" && export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1; rc=$?
  tail -3 "$O/pytest.log"
  [ $rc -eq 0 ] || exit $rc
fi
for B in ${SIZES:-65536 262144 1048576}; do
  for P in 0 0.01; do
    SW_FRAMED_TRACE=1 SW_TENANT_TRACE=1 timeout -k 10 400 python -u scripts/bench_tenant_path.py --devices 50000 --batch $B --batches 30 --warmup 4 \
      --via-bus --max-msgs $B --p-unregistered $P > "$O/tenant_${B}_${P}.log" 2>&1 || { tail -20 "$O/tenant_${B}_${P}.log"; exit 1; }
    tail -1 "$O/tenant_${B}_${P}.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["batch"], d["p_unregistered"], round(d["events_per_sec"]/1e6,1), "M/s", d["ms_per_batch"], "ms", d["mean_ms"], d.get("median_ms_second_half"), d["framed_trace_ms_per_batch"])'
  done
done
# 1M-payload, 200-batch soak through the bus: the producer outruns the engine, the protected raw
# topic must throttle it (0 records lost)
if [ "${SOAK:-1}" = "1" ]; then
  timeout -k 10 600 python -u scripts/bench_tenant_path.py --devices 50000 --batch 1048576 --batches 200 --warmup 4 \
    --via-bus --max-msgs 1048576 --no-alt-ids > "$O/soak_1m_200.log" 2>&1 || { tail -20 "$O/soak_1m_200.log"; exit 1; }
  tail -1 "$O/soak_1m_200.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("soak", round(d["events_per_sec"]/1e6,1), "M/s lost", d["raw_records_lost"], "waits", d["backpressure_waits"], "events", d["events"])'
fi
