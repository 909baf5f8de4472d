"""Probe: which engine serves a D2H copy (SDMA vs blit kernel) and at what rate; concurrency with a busy kernel."""
import ctypes
import sys
import time

import torch

import os; sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from sitewhere_amd._native import gpu  # noqa: E402
from sitewhere_amd.pipeline.gpu_engine import HostBuffer  # noqa: E402

N = 35 << 20
lib = gpu()
x = torch.randint(0, 255, (N,), dtype=torch.uint8, device="cuda")
h_torch = torch.empty(N, dtype=torch.uint8, pin_memory=True)
h_mapped = HostBuffer(lib, N)
s = torch.cuda.Stream()


def rate(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / reps
    return dt * 1e3, N / dt / 1e9


def torch_copy():
    with torch.cuda.stream(s):
        h_torch.copy_(x, non_blocking=True)


def abi_copy_mapped():
    lib.sw_copy_d2h(ctypes.c_void_p(h_mapped.host), ctypes.c_void_p(x.data_ptr()), N, ctypes.c_void_p(s.cuda_stream))


def abi_copy_torchpinned():
    lib.sw_copy_d2h(ctypes.c_void_p(h_torch.data_ptr()), ctypes.c_void_p(x.data_ptr()), N, ctypes.c_void_p(s.cuda_stream))


a = torch.randn(4096, 4096, device="cuda")


def busy():
    for _ in range(4):
        a.mul_(1.0001).add_(0.0001)


for name, fn in [("torch_pinned", torch_copy), ("abi_mapped", abi_copy_mapped), ("abi_torchpinned", abi_copy_torchpinned)]:
    ms, gbs = rate(fn)
    print(f"{name}: {ms:.3f} ms  {gbs:.1f} GB/s", flush=True)
ms_busy, _ = rate(busy)
print(f"busy alone: {ms_busy:.3f} ms")


def both():
    torch_copy()
    busy()


ms_both, _ = rate(both)
print(f"busy + concurrent torch D2H: {ms_both:.3f} ms")
hx = torch.empty(56 << 20, dtype=torch.uint8, pin_memory=True)
dx = torch.empty(56 << 20, dtype=torch.uint8, device="cuda")
s2 = torch.cuda.Stream()


def h2d():
    with torch.cuda.stream(s2):
        dx.copy_(hx, non_blocking=True)


ms, _ = rate(h2d)
print(f"H2D 56MB: {ms:.3f} ms  {56*1.048576/ms:.1f} GB/s")


def duplex():
    h2d()
    torch_copy()


ms, _ = rate(duplex)
print(f"H2D 56MB || D2H 35MB: {ms:.3f} ms")
