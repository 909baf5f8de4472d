#!/bin/bash
# GPU vs CPU header compare for several builds of the encoder (debugging a codegen-dependent mismatch)
for v in "" vB vC vD; do
  lib=sitewhere_amd/_lib/libswgpu${v:+_$v}.so
  echo "== variant ${v:-A} $lib"
  SW_GPU_LIB=$PWD/$lib timeout -k 10 120 python -u scripts/dbg/seg_hdr.py > gpurun_out/segvar_${v:-A}.log 2>&1 || exit $?
done
