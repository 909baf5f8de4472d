#!/bin/bash
# 64K-payload tenant path with the stack sampler (where the host threads spend the timed region)
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/tenant_sample && export TMPDIR=/tmp
SW_SAMPLE_STACKS=1 SW_TENANT_TRACE=1 timeout -k 10 300 python -u scripts/bench_tenant_path.py --devices 50000 --batch 65536 \
  --batches 300 --warmup 4 --via-bus --max-msgs 1048576 > gpurun_out/tenant_sample/run.log 2> gpurun_out/tenant_sample/stacks.err
