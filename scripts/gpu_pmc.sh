#!/bin/bash
# Hardware counters of the headline bench, one rocprofv3 pass per counter group (no --sys-trace):
#   pass 1 FETCH_SIZE (3 TCC counters), pass 2 WRITE_SIZE (2 TCC), pass 3 SQ/GRBM occupancy.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/pmc"
mkdir -p "$O" && cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 5 --warmup 2"
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$O/fetch" -o run -- python3 $B > "$O/fetch.log" 2>&1 && echo "fetch ok" &&
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$O/write" -o run -- python3 $B > "$O/write.log" 2>&1 && echo "write ok" &&
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d "$O/sq" -o run -- python3 $B > "$O/sq.log" 2>&1 && echo "sq ok"
