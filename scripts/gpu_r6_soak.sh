#!/bin/bash
# Round 6: steady-state soak of a gpu-columnar-1m tenant via the bus (1M devices, alternate ids, 0.5%
# unregistered, retention by rows bounded to the generational dedup filter), then the replay check.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r6_soak}
mkdir -p $O
export TMPDIR=/tmp
df -h /tmp > $O/df.txt 2>&1
nproc > $O/nproc.txt
timeout -k 10 ${SOAK_TIMEOUT:-1080} python -u scripts/soak_tenant.py --devices ${DEVICES:-1048576} \
    --phases ${PHASES:-3} --phase-s ${PHASE_S:-70} ${SOAK_ARGS} > $O/soak.json 2> $O/soak.err || { tail -30 $O/soak.err; exit 1; }
python - $O/soak.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print({k: d[k] for k in ("events_per_sec", "phase_events_per_sec", "first_minute_events_per_sec",
                         "last_minute_events_per_sec", "rechecks_per_payload", "setup_s", "trace")})
print("filter", d["filter"]["rotations"], d["filter"]["ids_ingested_per_capacity"], "store wraps", d["store"]["retention_wraps"])
print("replay", d["replay"])
PY
