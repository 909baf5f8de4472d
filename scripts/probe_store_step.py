"""Store-thread cost of one 1M-row columnar batch (payload build, event-management RPC, publish) in a
co-located instance, plus raw multi-threaded copy rates -- run on the GPU box's CPU share."""
import os, time, numpy as np, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import logging; logging.basicConfig(level=logging.ERROR)
from sitewhere_amd.assembly import SiteWhereInstance
from sitewhere_amd.models.columnar import OUT_REC
from sitewhere_amd.pipeline.engine_base import StepResult
sw = SiteWhereInstance().start(); sw.wait_for_tenant("default", 60)
tm = sw.api("TenantManagement")
sw.instance.system_user.run(lambda: tm.create_tenant({"token": "fast", "name": "fast", "configurationTemplateId": "gpu-columnar", "datasetTemplateId": "empty"}))
sw.wait_for_tenant("fast", 120)
ib = sw.tenant_engine("inbound-processing", "fast")
st = sw.tenant_engine("event-management", "fast").store
st.retention_rows = 8 << 20
bus = sw.instance.bus; t_out = sw.instance.naming.tenant_prefix("fast") + "inbound-enriched-batches"; bus.topic(t_out); bus.set_retention(t_out, 32 * (8 << 20))
rows = np.zeros(1 << 20, OUT_REC)
if len(sys.argv) > 1 and sys.argv[1] == "pinned":      # rows in torch pinned memory, as the engine returns them
    import torch
    pin = torch.zeros(rows.nbytes, dtype=torch.uint8).pin_memory()
    rows = pin.numpy().view(OUT_REC)
    print("rows in pinned host memory")
em = ib._em()
if "arena1" in sys.argv:        # every thread allocates from the main (brk) arena
    import ctypes
    print("M_ARENA_MAX=1:", ctypes.CDLL("libc.so.6").mallopt(-8, 1))


def loop():
  for k in range(24):
      n = (1 << 20) - (int(np.random.default_rng(k).integers(0, 50_000)) if "vary" in sys.argv else 0)
      res = StepResult(n_msgs=n, n_events=n, n_persisted=n, out=rows[:n], first_seq=k << 20)
      t0 = time.perf_counter(); p = ib.columnar_payload(res, 1); t1 = time.perf_counter()
      em.add_columnar_batch(p); t2 = time.perf_counter()
      bus.append_bytes(t_out, 0, p, ts=1); t3 = time.perf_counter()
      print(f"{k:2d} payload {1000*(t1-t0):.2f} rpc {1000*(t2-t1):.2f} publish {1000*(t3-t2):.2f}")


if "thread" in sys.argv:        # on a worker thread, like the tenant's store thread
    import threading
    th = threading.Thread(target=loop)
    th.start()
    th.join()
else:
    loop()

from sitewhere_amd._native import native
src = np.ones(32 << 20, np.uint8); dst = np.ones(32 << 20, np.uint8)
for th in (1, 2, 4, 8, 16):
    ts = []
    for _ in range(5):
        t = time.perf_counter(); native().sw_memcpy_mt(dst.ctypes.data, src.ctypes.data, src.nbytes, th); ts.append(time.perf_counter() - t)
    print(f"memcpy_mt 32 MB threads={th}: {1000*min(ts):.2f} ms (best of 5)")
print("cpus", len(os.sched_getaffinity(0)), "hw", os.cpu_count())
sw.stop()
