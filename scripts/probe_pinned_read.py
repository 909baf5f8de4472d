"""CPU read bandwidth of host buffers the GPU writes into: pageable, torch pinned, hipHostMalloc-mapped."""
import json
import sys
import os
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from sitewhere_amd._native import gpu  # noqa: E402
from sitewhere_amd.pipeline.gpu_engine import HostBuffer  # noqa: E402

n = 64 << 20
dev = torch.randint(0, 255, (n,), dtype=torch.uint8, device="cuda")
out = {}


def rd(name, arr):
    arr.copy()
    t = time.perf_counter()
    for _ in range(5):
        arr.copy()
    out[name] = round(5 * n / (time.perf_counter() - t) / 1e9, 2)


pin = torch.empty(n, dtype=torch.uint8).pin_memory()
pin.copy_(dev)
rd("torch_pinned_GBps", pin.numpy())
page = dev.cpu().numpy()
rd("pageable_GBps", page)
hb = HostBuffer(gpu(), n)
torch.cuda.synchronize()
rd("hip_mapped_GBps", hb.view(np.uint8, n))
t = time.perf_counter()
for _ in range(5):
    pin.copy_(dev)
torch.cuda.synchronize()
out["d2h_pinned_GBps"] = round(5 * n / (time.perf_counter() - t) / 1e9, 2)
t = time.perf_counter()
for _ in range(5):
    dev.cpu()
out["d2h_pageable_GBps"] = round(5 * n / (time.perf_counter() - t) / 1e9, 2)
print(json.dumps(out))
