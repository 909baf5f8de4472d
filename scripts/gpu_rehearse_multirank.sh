#!/bin/bash
# Rehearse the N>1 bench path on a one-GPU box: N ranks share GPU 0 and exchange through gloo
# (RCCL refuses two ranks on one device).  Real kernels, real pipelined exchange code path.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/rehearse
cd "$R" && mkdir -p $O
export SW_SHARED_DEVICE=1 SW_DIST_BACKEND=gloo
for n in ${NS:-2 4}; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --steps ${STEPS:-10} --warmup ${WARM:-3} \
    --msgs ${MSGS:-262144} --devices ${DEVS:-262144} --store $((1 << 24)) > $O/n$n.log 2>&1 || { echo "n=$n failed"; tail -20 $O/n$n.log; exit 1; }
  tail -1 $O/n$n.log | cut -c1-220
done
