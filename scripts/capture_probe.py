"""Does a legacy-null-stream op issued by another thread while this process captures a hipGraph on
a torch stream (HIP thread-local capture mode, as sw_graph_capture_process) run, fail, or land in
the graph?  Thread B index_copy_'s a marker into a table while thread A holds a capture open."""
import ctypes
import threading
import time

import torch

hip = ctypes.CDLL("libamdhip64.so")
dev = torch.device("cuda:0")
cap = torch.cuda.Stream(dev)
flags = ctypes.c_uint()
hip.hipStreamGetFlags(ctypes.c_void_p(cap.cuda_stream), ctypes.byref(flags))
print("capture stream flags", flags.value, "(1 = non-blocking)")
x = torch.zeros(1 << 20, device=dev)
table = torch.zeros(16, 4, dtype=torch.int64, device=dev)
torch.cuda.synchronize()
res = {}


def writer():
    time.sleep(0.05)                      # inside A's capture window
    try:
        idx = torch.tensor([3], device=dev)
        rows = torch.full((1, 4), 7, dtype=torch.int64, device=dev)
        table.index_copy_(0, idx, rows)
        torch.cuda.current_stream(dev).synchronize()
        res["b"] = "ok"
    except Exception as e:                # noqa: BLE001
        res["b"] = repr(e)


g = ctypes.c_void_p()
ex = ctypes.c_void_p()
t = threading.Thread(target=writer)
with torch.cuda.stream(cap):
    rc = hip.hipStreamBeginCapture(ctypes.c_void_p(cap.cuda_stream), 1)   # 1 = thread-local
    t.start()
    for _ in range(200):
        x.mul_(1.0001)
    time.sleep(0.2)
    rc2 = hip.hipStreamEndCapture(ctypes.c_void_p(cap.cuda_stream), ctypes.byref(g))
    t.join()
print("begin", rc, "end", rc2, "writer", res.get("b"))
torch.cuda.synchronize()
print("row 3 after capture:", table[3].tolist())
if rc2 == 0 and g.value:
    rc3 = hip.hipGraphInstantiate(ctypes.byref(ex), g, None, None, 0)
    table.zero_()
    torch.cuda.synchronize()
    hip.hipGraphLaunch(ex, ctypes.c_void_p(cap.cuda_stream))
    torch.cuda.synchronize()
    n = ctypes.c_size_t()
    hip.hipGraphGetNodes(g, None, ctypes.byref(n))
    print("instantiate", rc3, "graph nodes", n.value, "row 3 after a replay:", table[3].tolist())
