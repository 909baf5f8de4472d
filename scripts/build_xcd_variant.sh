#!/bin/bash
# Build libswgpu_xcd.so: the same kernels with the XCD-aware block-id remap (SW_XCD_REMAP=1).
# Load it instead of the default library with SW_GPU_LIB=<path>.
set -e
R="$(cd "$(dirname "$0")/.." && pwd)"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -DSW_XCD_REMAP=1 -I"$R/csrc/include" \
  -o "$R/sitewhere_amd/_lib/libswgpu_xcd.so" "$R"/csrc/hip/*.hip -lhsa-runtime64
echo "$R/sitewhere_amd/_lib/libswgpu_xcd.so"
