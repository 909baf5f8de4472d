#!/bin/bash
# A multi-process instance on one node without containers: infra, the global and multitenant
# services, and one inbound-processing replica per visible GPU (SITEWHERE_GPU_DEVICE), each its own
# process.  Logs go to $LOGS.  Stop with Ctrl-C: the script ends the process group it started.
#   SITEWHERE_JWT_SECRET=... deploy/run_node.sh [n_gpus]
set -u
cd "$(dirname "$0")/.."
: "${SITEWHERE_JWT_SECRET:?set a shared JWT secret}"
export SITEWHERE_JWT_SECRET HSA_ENABLE_IPC_MODE_LEGACY=0
N=${1:-$(python -c "import torch; print(torch.cuda.device_count())")}
INFRA=127.0.0.1:9092
LOGS=${LOGS:-/tmp/sitewhere-logs}
mkdir -p "$LOGS"
trap 'kill 0' INT TERM EXIT
python -m sitewhere_amd.serve infra --port 9092 --data "${DATA:-/tmp/sitewhere-data}" > "$LOGS/infra.log" 2>&1 &
sleep 2
python -m sitewhere_amd.serve service instance-management tenant-management user-management web-rest \
  --infra $INFRA --rest-port 8080 > "$LOGS/global.log" 2>&1 &
python -m sitewhere_amd.serve service event-sources --infra $INFRA > "$LOGS/event-sources.log" 2>&1 &
python -m sitewhere_amd.serve service device-management event-management asset-management device-registration \
  device-state rule-processing outbound-connectors command-delivery batch-operations schedule-management \
  label-generation streaming-media event-search --infra $INFRA > "$LOGS/multitenant.log" 2>&1 &
for ((g = 0; g < N; g++)); do
  SITEWHERE_GPU_DEVICE=$g python -m sitewhere_amd.serve service inbound-processing --infra $INFRA \
    > "$LOGS/inbound-gpu$g.log" 2>&1 &
done
echo "instance starting: REST http://127.0.0.1:8080/sitewhere/api, $N inbound-processing GPU replica(s); logs in $LOGS"
wait
