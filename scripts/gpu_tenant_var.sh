R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/tenant_var; cd "$R" && mkdir -p $O
b=1048576
for th in 0 4; do
SW_MEMCPY_THREADS=$th SW_TENANT_TRACE=1 timeout -k 10 300 python scripts/bench_tenant_path.py --devices 20000 --batch $b --batches 60 --max-msgs $b --via-bus --store-retention $(( 8 * b )) > $O/ret_th$th.log 2>&1 && tail -1 $O/ret_th$th.log || exit 1
done
