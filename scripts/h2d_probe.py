"""Host time of the tenant's H2D enqueue (submit_framed): a 1M-payload raw record on the bus is a
pinned buffer; torch.frombuffer views of it are copied to HBM with non_blocking=True.  Reports
whether torch sees the view as pinned and the host time of each copy call (an async enqueue takes
microseconds; a staged synchronous copy takes the transfer time)."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from sitewhere_amd.pipeline.bus_io import RawBatchRecord, parse_raw_batch  # noqa: E402
from sitewhere_amd.pipeline.fleet import FleetSpec, gen_payloads  # noqa: E402
from sitewhere_amd.pipeline.framing import varint_lengths  # noqa: E402

spec = FleetSpec(prefix="dev-", n_devices=1 << 20, with_alternate_id=True)
raw, off = gen_payloads(spec, 1 << 20, 1_700_000_000_000, seed=3)
rec = RawBatchRecord(raw[:int(off[-1])], varint_lengths(off), len(off) - 1, pinned=True)
b = parse_raw_batch(rec.buf.numpy()[:rec.value_len])
dev = torch.empty(len(b.payload) + 4096, dtype=torch.uint8, device="cuda")
s = torch.cuda.Stream()
out = {"bytes": len(b.payload)}
for name, src in (("frombuffer", lambda: torch.frombuffer(b.payload, dtype=torch.uint8)),
                  ("record_tensor", lambda: rec.buf[:len(b.payload)])):
    t = src()
    out[f"{name}_is_pinned"] = bool(t.is_pinned())
    ts = []
    for _ in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            dev[:t.numel()].copy_(t, non_blocking=True)
        ts.append((time.perf_counter() - t0) * 1e3)
        torch.cuda.synchronize()
    out[f"{name}_enqueue_ms"] = [round(x, 3) for x in ts]
print(json.dumps(out))
