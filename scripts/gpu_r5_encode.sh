#!/bin/bash
# k_seg_encode geometry variants: the built-in encoder and swseg.hip builds with other
# SW_SEG_SBLK / SW_SEG_MIN_WAVES (sitewhere_amd/_lib/variants/, built on the CPU beforehand), 1M rows
# with strings, each variant's block checked byte for byte against the built-in one.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r5_encode
export TMPDIR=/tmp
out=gpurun_out/r5_encode/seg_variants_b.jsonl
: > $out
timeout -k 10 120 python -u scripts/bench_seg_encode.py --n 1048576 --reps 20 --stamps >> $out 2> gpurun_out/r5_encode/err.log || exit $?
for v in sitewhere_amd/_lib/variants/libseg_*.so; do
  timeout -k 10 120 python -u scripts/bench_seg_encode.py --n 1048576 --reps 20 --stamps --lib $v >> $out 2>> gpurun_out/r5_encode/err.log || exit $?
done
cat $out
timeout -k 10 180 python -u scripts/bench_dedup_micro.py > gpurun_out/r5_encode/dedup_micro.jsonl 2>> gpurun_out/r5_encode/err.log || exit $?
cat gpurun_out/r5_encode/dedup_micro.jsonl
