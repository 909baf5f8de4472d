"""World-8 rehearsal on one MI355X: eight engines of one 8-GPU job, in one process
on one GPU, at the bench's N=8 shapes.

Each rank's engine holds the whole replicated registry (8 x --devices), decodes its own 1M-payload
batch and partitions the records by owner into the per-destination slabs of the all-to-all re-key
(``sw_phase_partition``); the exchange is done by device-to-device copies of the slabs and their
string slabs (the loopback of ``tests/test_multirank.py``, what ``phase_exchange`` moves over RCCL);
every rank then unpacks and processes what it owns.  The ranks run one after the other, so each
rank's kernels have the GPU alone: per rank, the decode+partition and unpack+process times (HIP
events on the compute stream) and the bytes its slabs send to the other seven ranks.  The same
batches through a world-1 engine give the N=1 step for comparison.  Prints one JSON line.

    python scripts/world8_rehearsal.py --msgs 1048576 --devices 1048576 --steps 4
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--msgs", type=int, default=1 << 20, help="payloads per rank per step")
    ap.add_argument("--devices", type=int, default=1 << 20, help="registered devices per rank")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--filter-ids", type=int, default=1 << 26, help="dedup filter ids per generation per rank")
    a = ap.parse_args()
    import torch
    from sitewhere_amd.models.columnar import STR_REF, WIRE_REC
    from sitewhere_amd.pipeline.config import EngineConfig
    from sitewhere_amd.pipeline.fleet import FleetSpec, fingerprints, gen_payloads, gen_tokens
    from sitewhere_amd.pipeline.gpu_engine import GpuInboundEngine
    W = a.world
    n_total = a.devices * W
    t0 = time.time()
    heap, offs = gen_tokens("dev-", 0, n_total)
    lo, hi = fingerprints(heap, offs)

    def config(world, rank):
        return EngineConfig(max_msgs=a.msgs, rec_cap=a.msgs + 4096, gen_cap=max(1 << 16, a.msgs // 2),
                            max_devices=int(n_total * 1.1) + 1024, max_assignments=int(n_total * 1.1) + 1024,
                            store_cap=1 << 22, dedup_slots=1 << 22, name_slots=1 << 12, rank=rank, world=world,
                            dedup_filter_ids=a.filter_ids, dedup_filter_gens=4,
                            state_slots=2 * (16 + 4 + 16) * int(a.devices * 1.1))

    def engine(world, rank):
        e = GpuInboundEngine(config(world, rank), device="cuda:0")
        d = e.register_devices(lo, hi)
        e.set_assignments(d, d, customer=d % 97, area=d % 31, asset=d % 1009)
        return e

    engines = [engine(W, r) for r in range(W)]
    one = engine(1, 0)
    now0 = int(time.time() * 1000)
    batches = []                                   # per step, per rank: (raw, offs, n) on the device
    n_steps = a.warmup + a.steps
    for k in range(n_steps):                       # every (step, rank) batch distinct: no replays
        row = []
        for r in range(W):
            spec = FleetSpec(prefix="dev-", n_devices=n_total, p_location=0.25, p_alert=0.05, p_unregistered=0.005,
                             n_names=16, with_alternate_id=True, lat0=33.0, lon0=-85.0, span_deg=2.0, p_meta=0.1,
                             alt_base=r << 24)
            raw, off = gen_payloads(spec, a.msgs, now0 - 30_000, seed=1 + 1000 * k + r)
            raw = np.concatenate([raw, np.zeros(64, np.uint8)])
            row.append((torch.from_numpy(raw).cuda(), torch.from_numpy(off.view(np.int32)).cuda(), len(off) - 1))
        batches.append(row)
    setup_s = time.time() - t0
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    per_rank = {r: {"decode_partition_ms": [], "unpack_process_ms": [], "exchange_bytes": []} for r in range(W)}
    n1 = []
    loop_ms = []
    for k in range(n_steps):
        now = now0 + 1000 * k
        marks = []
        for r, e in enumerate(engines):
            rd, od, n = batches[k][r]
            e0, e1 = ev(), ev()
            e0.record()
            e.prepare(rd, od, n, now)
            e.phase_decode()
            e1.record()
            marks.append((e0, e1))
        torch.cuda.synchronize()
        t_x = time.perf_counter()
        rec_b, sp_b = WIRE_REC.itemsize, STR_REF.itemsize
        sent = [0] * W
        for q in range(W):
            for r in range(W):
                engines[q].recv_slab(r).copy_(engines[r].send_slab(q))
                engines[q].t["recv_cnt"][r] = engines[r].send_count(q)
            engines[q].loopback_strings(engines)
        torch.cuda.synchronize()
        loop_ms.append((time.perf_counter() - t_x) * 1e3)
        for r, e in enumerate(engines):
            p = e._last_send_par
            cnt = e.send_cnts[p].cpu().numpy().astype(np.int64)
            scnt = e.send_str_cnts[p].cpu().numpy().astype(np.int64) if e.cfg.str_cap else np.zeros(W, np.int64)
            sent[r] = int(sum(cnt[q] * (rec_b + sp_b) + scnt[q] for q in range(W) if q != r))
        pmarks = []
        for e in engines:
            e2, e3 = ev(), ev()
            e2.record()
            e.phase_process()
            e3.record()
            pmarks.append((e2, e3))
        torch.cuda.synchronize()
        # N=1: one rank's payload volume through a world-1 engine
        rd, od, n = batches[k][0]
        f0, f1 = ev(), ev()
        f0.record()
        one.prepare(rd, od, n, now)
        one.phase_decode()
        one.phase_process()
        f1.record()
        torch.cuda.synchronize()
        if k >= a.warmup:
            for r in range(W):
                per_rank[r]["decode_partition_ms"].append(marks[r][0].elapsed_time(marks[r][1]))
                per_rank[r]["unpack_process_ms"].append(pmarks[r][0].elapsed_time(pmarks[r][1]))
                per_rank[r]["exchange_bytes"].append(sent[r])
            n1.append(f0.elapsed_time(f1))
    stats = [e.stats_dict() for e in engines]
    s1 = one.stats_dict()
    rank_ms = [float(np.mean(np.array(per_rank[r]["decode_partition_ms"]) + np.array(per_rank[r]["unpack_process_ms"])))
               for r in range(W)]
    n1_ms = float(np.mean(n1))
    out = {"bench": "world8_rehearsal", "world": W, "payloads_per_rank_step": a.msgs, "devices_per_rank": a.devices,
           "steps": a.steps, "setup_s": round(setup_s, 1),
           "n1_step_kernels_ms": round(n1_ms, 3),
           "rank_step_kernels_ms": [round(x, 3) for x in rank_ms],
           "max_rank_vs_n1": round(max(rank_ms) / n1_ms, 3),
           "per_rank": {r: {k2: [round(float(x), 3) for x in v] for k2, v in d.items()} for r, d in per_rank.items()},
           "exchange_bytes_per_rank_step": int(np.mean([np.mean(per_rank[r]["exchange_bytes"]) for r in range(W)])),
           "loopback_copy_ms": round(float(np.mean(loop_ms[a.warmup:])), 3),
           "events": {"world8_persisted": int(sum(s["persisted"] for s in stats)),
                      "world8_events": int(sum(s["events"] for s in stats)),
                      "n1_persisted": int(s1["persisted"]), "n1_events": int(s1["events"]),
                      "world8_duplicates": int(sum(s["duplicates"] for s in stats)),
                      "world8_unregistered": int(sum(s["unregistered"] for s in stats))}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
