"""Which HIP stream a thread's torch "current stream" is: the main thread's and a worker thread's
(a per-thread default stream would not order a worker's table writes before the main thread's steps)."""
import threading

import torch

out = {}


def probe(name):
    out[name] = hex(torch.cuda.current_stream().cuda_stream)


probe("main")
t = threading.Thread(target=probe, args=("worker",))
t.start()
t.join()
print(out)
