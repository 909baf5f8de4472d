#!/bin/bash
# Same-box comparison: MI355X engine vs the native CPU engine (16-core share) vs the per-event design,
# plus the config #1 tenant path on the GPU engine.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/cmp
cd "$R" && export TMPDIR=/tmp && mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && tail -1 $O/pytest_gpu.log &&
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > $O/bench_gpu.log 2>&1 && tail -1 $O/bench_gpu.log | cut -c1-150 &&
timeout -k 10 400 env SW_CPU_ENGINE_THREADS=16 python bench.py --engine cpu --steps 8 --warmup 3 > $O/bench_cpu16.log 2>&1 && tail -1 $O/bench_cpu16.log | cut -c1-150 &&
timeout -k 10 400 python scripts/bench_reference_config.py --path engine --events 2000000 --batch 65536 > $O/config1_engine_gpu_64k.log 2>&1 && tail -1 $O/config1_engine_gpu_64k.log &&
timeout -k 10 400 python scripts/bench_reference_config.py --path engine --events 4000000 --batch 262144 > $O/config1_engine_gpu_256k.log 2>&1 && tail -1 $O/config1_engine_gpu_256k.log &&
timeout -k 10 300 python scripts/bench_reference_config.py --replicas 0 --events 1000 --paced 1000 > $O/config1_inproc.log 2>&1 && tail -1 $O/config1_inproc.log
