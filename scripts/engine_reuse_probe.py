"""Engine lifecycle probe: GPU engines created one after another in one process (the caching
allocator hands each the memory its predecessors freed), devices registered from a second thread
while the first steps batches, then a batch from a registered device must persist in full.
Prints one JSON line per engine: persisted vs expected and the step's counters."""
import gc
import json
import sys
import threading
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from sitewhere_amd.models import wire  # noqa: E402
from sitewhere_amd.pipeline.bus_io import RawBatch  # noqa: E402
from sitewhere_amd.pipeline.config import EngineConfig  # noqa: E402
from sitewhere_amd.pipeline.fleet import fingerprint_str, pack_messages  # noqa: E402
from sitewhere_amd.pipeline.gpu_engine import GpuInboundEngine  # noqa: E402

COLUMNAR = {"max_msgs": 1 << 18, "max_devices": 65536, "max_assignments": 65536, "store_cap": 1 << 22,
            "dedup_slots": 1 << 24, "gen_cap": 32768, "dedup_filter_ids": (1 << 28) - (1 << 21)}


def batch(msgs):
    raw, offs = pack_messages(msgs)
    return RawBatch(len(offs) - 1, int(offs[-1]), raw, offs=offs)


def one(k: int, cap: dict, threaded: bool, encode: bool) -> dict:
    e = GpuInboundEngine(EngineConfig.small(**cap), device="cuda:0")
    if encode:
        e.encode_blocks, e.block_boot = True, 1
    now = 1_700_000_000_000
    toks = [f"probe-{k}-{i:03d}" for i in range(24)]

    def register():
        for i, t in enumerate(toks):
            lo, hi = fingerprint_str(t)
            e.register_devices(np.array([lo], np.uint64), np.array([hi], np.uint64), np.array([i], np.int32))
            e.set_assignments([i], [i], active=[1])
            time.sleep(0.002)

    noise = batch([wire.measurements(f"stranger-{j}", {"v": 1.0}) for j in range(50)])
    if threaded:
        th = threading.Thread(target=register)
        th.start()
        while th.is_alive():
            e.step_framed(noise, now)
        th.join()
    else:
        register()
    before = e.stats_dict()
    msgs = [wire.measurements(toks[3], {"v": float(i)}, event_date=now + i) for i in range(200)]
    msgs.append(wire.measurements("nobody", {"v": 1.0}))
    res = e.step_framed(batch(msgs), now + 1000)
    after = e.stats_dict()
    torch.cuda.synchronize()
    d = {k2: after[k2] - before.get(k2, 0) for k2 in after if after[k2] != before.get(k2, 0)}
    out = {"engine": k, "columnar_caps": cap is COLUMNAR, "threaded": threaded, "encode": encode,
           "persisted": int(res.n_persisted), "expected": 200, "step_counters": d}
    del e, res
    gc.collect()
    return out


if __name__ == "__main__":
    bad = 0
    for k in range(8):
        cap = COLUMNAR if k % 2 == 0 else {}
        r = one(k, cap, threaded=k % 4 < 2, encode=k % 3 != 2)
        bad += r["persisted"] != r["expected"]
        print(json.dumps(r), flush=True)
    print(json.dumps({"engines": 8, "short": bad}), flush=True)
