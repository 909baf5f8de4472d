#!/bin/bash
# Round 5: where the gpu-columnar tenant path with alternate ids spends its time -- sampled Python
# stacks of every thread, then the GPU kernels of the same run shape under rocprofv3.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${1:-r5_tenant_diag}"
mkdir -p "$O" && cd "$R" && export TMPDIR=/tmp
ARGS="--devices 50000 --batch 65536 --batches 400 --warmup 4 --via-bus --max-msgs 262144"
SW_SAMPLE_STACKS=1 SW_TENANT_TRACE=1 SW_FRAMED_TRACE=1 timeout -k 10 300 python -u scripts/bench_tenant_path.py $ARGS \
    > "$O/alt_stacks.log" 2> "$O/alt_stacks.err" || exit 1
P=/tmp/sw_tdiag_prof
summ() {   # the kernel table and one step's dispatches; the database itself stays on the box
  python "$R/scripts/rocpd_summary.py" "$P/$1/run_results.db" --steps 404 --md "$O/$1_kernels.md" > /dev/null
  python "$R/scripts/step_dispatches.py" "$P/$1/run_results.db" --step 200 > "$O/$1_dispatches.md" 2>&1 || true
  rm -rf "$P/$1"
}
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$P/alt" -o run -- \
    python -u "$R/scripts/bench_tenant_path.py" $ARGS > "$O/alt_prof.log" 2> "$O/alt_prof.err" || exit 1
summ alt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$P/noalt" -o run -- \
    python -u "$R/scripts/bench_tenant_path.py" $ARGS --no-alt-ids > "$O/noalt_prof.log" 2> "$O/noalt_prof.err" || exit 1
summ noalt
