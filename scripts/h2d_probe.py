"""PCIe H2D probe: which copy mechanism moves a bench-sized raw batch (85 MB) fastest on this box.
torch copy_ on one stream vs split over streams vs explicit SDMA engines (sw_sdma_h2d)."""
import ctypes
import json
import time

import torch

from sitewhere_amd._native import gpu

lib = gpu()
N = 85 << 20
dev = torch.device("cuda:0")
host = torch.empty(N, dtype=torch.uint8).pin_memory()
host.random_(0, 255)
d = torch.empty(N, dtype=torch.uint8, device=dev)
res = {}


def bench(name, fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / reps
    res[name] = {"ms": round(dt * 1e3, 3), "GBps": round(N / dt / 1e9, 1)}
    print(name, res[name], flush=True)


s1, s2, s3, s4 = (torch.cuda.Stream(dev) for _ in range(4))


def one():
    with torch.cuda.stream(s1):
        d.copy_(host, non_blocking=True)


def split(k, streams):
    c = N // k

    def f():
        for i in range(k):
            with torch.cuda.stream(streams[i % len(streams)]):
                d[i * c:(i + 1) * c].copy_(host[i * c:(i + 1) * c], non_blocking=True)
    return f


def sdma(engines):
    def f():
        k = len(engines)
        c = N // k
        sigs = []
        for i, e in enumerate(engines):
            sig = ctypes.c_uint64(0)
            rc = lib.sw_sdma_h2d(ctypes.c_void_p(d.data_ptr() + i * c), ctypes.c_void_p(host.data_ptr() + i * c),
                                 c, e, ctypes.byref(sig))
            assert rc == 0, rc
            sigs.append(sig.value)
        for sg in sigs:
            assert lib.sw_sdma_wait(ctypes.c_uint64(sg)) == 0
    return f


bench("torch_1stream", one)
bench("torch_split2_2streams", split(2, [s1, s2]))
bench("torch_split4_4streams", split(4, [s1, s2, s3, s4]))
for engs in ([0], [1], [1, 2], [1, 2, 3, 4]):
    try:
        bench(f"sdma_engines_{'_'.join(map(str, engs))}", sdma(engs))
    except AssertionError as e:
        print("sdma", engs, "failed", e)
# H2D while a D2H of 17 MB runs (full duplex check)
dd = torch.empty(17 << 20, dtype=torch.uint8, device=dev)
hh = torch.empty(17 << 20, dtype=torch.uint8).pin_memory()


def duplex():
    with torch.cuda.stream(s2):
        hh.copy_(dd, non_blocking=True)
    one()


bench("torch_h2d_with_d2h", duplex)
print(json.dumps(res))
