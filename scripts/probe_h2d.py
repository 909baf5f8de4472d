"""Probe: H2D bandwidth of the 56 MB payload batch -- HIP runtime copy vs explicit copy engines,
one engine vs the batch split across several engines, and H2D || D2H duplex."""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from sitewhere_amd._native import gpu  # noqa: E402

lib = gpu()
N = 56 << 20
hx = torch.randint(0, 255, (N,), dtype=torch.uint8).pin_memory()
dx = torch.empty(N, dtype=torch.uint8, device="cuda")
s = torch.cuda.Stream()


def rate(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / reps
    return dt * 1e3, N / dt / 1e9


def torch_h2d():
    with torch.cuda.stream(s):
        dx.copy_(hx, non_blocking=True)
    s.synchronize()


def engines_h2d(engines):
    def fn():
        k = len(engines)
        chunk = (N // k + 4095) & ~4095
        sigs = []
        for i, e in enumerate(engines):
            off = i * chunk
            n = min(chunk, N - off)
            if n <= 0:
                break
            h = ctypes.c_uint64()
            rc = lib.sw_sdma_h2d(ctypes.c_void_p(dx.data_ptr() + off), ctypes.c_void_p(hx.data_ptr() + off), n, e,
                                 ctypes.byref(h))
            if rc:
                raise RuntimeError(f"sw_sdma_h2d engine {e} rc={rc}")
            sigs.append(h.value)
        for h in sigs:
            lib.sw_sdma_wait(h)
    return fn


ms, gbs = rate(torch_h2d)
print(f"torch H2D 56MB: {ms:.3f} ms {gbs:.1f} GB/s", flush=True)
assert torch.equal(dx.cpu(), hx)
for engines in ([0], [1], [2], [1, 2], [1, 2, 3, 4], [1, 2, 3, 4, 5, 6, 7, 8]):
    try:
        dx.zero_()
        ms, gbs = rate(engines_h2d(engines))
        ok = torch.equal(dx.cpu(), hx)
        print(f"hsa H2D engines={engines}: {ms:.3f} ms {gbs:.1f} GB/s correct={ok}", flush=True)
    except Exception as ex:  # noqa: BLE001
        print(f"hsa H2D engines={engines}: failed {ex}", flush=True)
h_out = torch.empty(32 << 20, dtype=torch.uint8, pin_memory=True)
d_out = torch.randint(0, 255, (32 << 20,), dtype=torch.uint8, device="cuda")


def duplex():
    h = ctypes.c_uint64()
    lib.sw_sdma_copy(ctypes.c_void_p(h_out.data_ptr()), ctypes.c_void_p(d_out.data_ptr()), 32 << 20, 0, ctypes.byref(h))
    torch_h2d()
    lib.sw_sdma_wait(h.value)


ms, _ = rate(duplex)
print(f"torch H2D 56MB || hsa D2H 32MB: {ms:.3f} ms", flush=True)
