#!/usr/bin/env python3
"""Headline benchmark: device events/sec through the SiteWhere inbound pipeline on MI355X.

Reference headline (BASELINE.json): "device events/sec through the Kafka pipeline" --
decode -> inbound validation -> event persistence -> enrichment -> consumers
(device state, rule processing, outbound connectors).  The reference publishes no
number, so ``vs_baseline`` is null.

One step = one micro-batch of ``--msgs`` protobuf device payloads per GPU, run end to end:
  raw batch produced to the raw-payload topic of the native commit log (zero-copy, pinned record)
  -> consumed in place -> H2D of the raw wire bytes straight from the topic -> GPU decode -> [N>1: owner partition + RCCL
  all-to-all re-keying by device token, the analogue of Kafka key partitioning] -> registry
  lookup + assignment validation -> alternate-id dedup -> persist into the HBM event store
  with enrichment -> device-state merge -> zone-test rules (point-in-polygon, generated alerts
  persisted too) -> presence scan -> D2H of every enriched event into a pinned record published
  to the enriched-batch topic -> consumer offset commit (``--no-bus``: pinned batches in, host ring out).
Weak scaling: per-GPU payloads and per-GPU device shard are fixed as N grows.

Launch: ``python bench.py --gpus 1 --steps 200 --warmup 20`` or under torch.distributed.run
for N > 1 (one rank per GPU, RCCL).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np


def parse():
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)   # ~0.2 s timed at N=1: steady state, not warm-up
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--msgs", type=int, default=1 << 20, help="payloads per GPU per step")
    ap.add_argument("--devices", type=int, default=1 << 20, help="registered devices per GPU")
    ap.add_argument("--mx-per-msg", type=int, default=1)
    ap.add_argument("--batches", type=int, default=4, help="distinct pre-generated batches to cycle")
    ap.add_argument("--zones", type=int, default=16)
    ap.add_argument("--store", type=int, default=1 << 27, help="HBM event-store capacity per GPU (events)")
    ap.add_argument("--engine", choices=["gpu", "cpu", "oracle"], default="gpu",
                    help="gpu: MI355X kernels; cpu: native multi-threaded C++ engine; oracle: Python reference")
    ap.add_argument("--framing", choices=["varint", "offsets"], default="varint",
                    help="raw-batch framing on the wire to the GPU (varint lengths or u32 offsets)")
    ap.add_argument("--no-outbound", action="store_true", help="(diagnostic) skip the D2H outbound copy")
    ap.add_argument("--bus", action=argparse.BooleanOptionalAction, default=True,
                    help="GPU engine: consume raw batches from, and publish enriched batches to, commit-log "
                         "topics in place (pipeline/bus_io.py); --no-bus feeds pinned batches directly")
    return ap.parse_args()


def zone_polys(n, lat0, lon0, span, rng):
    from sitewhere_amd.pipeline.engine_base import Zone, ZoneTest
    zones, tests = [], []
    for z in range(n):
        cx, cy = lat0 + rng.uniform(0.1, 0.9) * span, lon0 + rng.uniform(0.1, 0.9) * span
        r = span * 0.08
        k = 32
        ang = np.sort(rng.uniform(0, 2 * np.pi, k))
        rad = r * rng.uniform(0.6, 1.0, k)
        verts = [(cx + rad[i] * np.cos(ang[i]), cy + rad[i] * np.sin(ang[i])) for i in range(k)]
        zones.append(Zone(f"zone-{z}", verts))
        tests.append(ZoneTest(f"zone-{z}", "inside", f"zone.{z}.enter", 2, "entered restricted zone"))
    return zones, tests


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from sitewhere_amd.parallel.sharding import init_distributed, shard_mask

    use_gpu = args.engine == "gpu"
    rank, local, world, _ = init_distributed(use_gpu)
    from sitewhere_amd.pipeline.config import EngineConfig
    from sitewhere_amd.pipeline.fleet import FleetSpec, gen_payloads, gen_tokens, fingerprints
    from sitewhere_amd.pipeline.framing import varint_lengths

    n_total_dev = args.devices * world
    spec = FleetSpec(prefix="dev-", n_devices=n_total_dev, p_location=0.25, p_alert=0.05, p_unregistered=0.0,
                     mx_per_msg=args.mx_per_msg, n_names=16, with_alternate_id=False,
                     lat0=33.0, lon0=-85.0, span_deg=2.0)
    cfg = EngineConfig(max_msgs=args.msgs, rec_cap=args.msgs * args.mx_per_msg + 4096,
                       gen_cap=max(1 << 16, args.msgs // 2), max_devices=int(args.devices * 1.1) + 1024,
                       max_assignments=int(args.devices * 1.1) + 1024, store_cap=args.store,
                       dedup_slots=1 << 20, name_slots=1 << 12, rank=rank, world=world,
                       # (assignment, name) state map: 16 measurement names + 4 alert types + zone alerts per device
                       state_slots=2 * (16 + 4 + args.zones) * int(args.devices * 1.1),
                       presence_missing_ms=8 * 3600 * 1000)
    if use_gpu:
        from sitewhere_amd.pipeline.gpu_engine import GpuInboundEngine, PipelinedRunner
        eng = GpuInboundEngine(cfg, device=torch.device("cuda", local), group=None)
    elif args.engine == "cpu":
        from sitewhere_amd.pipeline.native_engine import NativeCpuEngine
        eng = NativeCpuEngine(cfg)
    else:
        from sitewhere_amd.pipeline.cpu_engine import CpuInboundEngine
        eng = CpuInboundEngine(cfg)

    # ---- registry shard: the devices this rank owns (owner = fp_hi >> 32 mod world)
    t0 = time.time()
    heap, offs = gen_tokens("dev-", 0, n_total_dev)
    lo, hi = fingerprints(heap, offs)
    mine = shard_mask(hi, world, rank)
    lo, hi = lo[mine], hi[mine]
    dev = eng.register_devices(lo, hi)
    n_dev = len(dev)
    eng.set_assignments(dev, dev, customer=dev % 97, area=dev % 31, asset=dev % 1009)
    rng = np.random.default_rng(1234)
    zones, tests = zone_polys(args.zones, spec.lat0, spec.lon0, spec.span_deg, rng)
    eng.set_zone_rules(zones, tests)
    # ---- pre-generated synthetic raw batches (this rank's ingest stream)
    now0 = int(time.time() * 1000)
    batches = []
    for b in range(args.batches):
        raw, offs_b = gen_payloads(spec, args.msgs, now0 - 30_000, seed=1 + rank * 1000 + b)
        raw = np.concatenate([raw, np.zeros(64, np.uint8)])
        if use_gpu:
            # wire framing: payload bytes + a varint length per payload (offsets are rebuilt on the GPU)
            lens = varint_lengths(offs_b) if args.framing == "varint" else None
            batches.append((torch.from_numpy(raw).pin_memory(), torch.from_numpy(offs_b.view(np.int32)).pin_memory(),
                            raw, offs_b, None if lens is None else torch.from_numpy(lens).pin_memory()))
        else:
            batches.append((None, None, raw, offs_b, None))
    setup_s = time.time() - t0
    max_raw = max(int(b[2].size) for b in batches)

    def barrier():
        if world > 1:
            dist.barrier()
        if use_gpu:
            torch.cuda.synchronize()

    bus_stats = None
    if use_gpu and args.bus and args.framing == "varint":
        # Through the bus: each step the producer side hands raw batch k to the raw-payload topic
        # (zero-copy: the record is the pinned buffer), the engine's consumer reads it in place and
        # DMAs it to HBM, and the step's enriched rows are DMA'd into a pinned record published to
        # the enriched-batch topic.  Consumer offsets are committed once a batch's rows are out.
        from collections import deque

        from sitewhere_amd.bus.log import EventBus
        from sitewhere_amd.bus.naming import TopicNaming
        from sitewhere_amd.pipeline.bus_io import OutboundPublisher, RawBatchRecord, raw_view
        bus = EventBus(None, default_partitions=1)
        prefix = TopicNaming("sitewhere", f"bench-rank{rank}").tenant_prefix("default")
        t_raw, t_out = prefix + "event-source-raw-payloads", prefix + "inbound-enriched-batches"
        group = prefix + "inbound-processing.raw-payload-consumers"
        bus.topic(t_raw, 1)
        bus.set_retention(t_raw, 4 * max_raw)
        records = [RawBatchRecord(b[2][:int(b[3][-1])], b[4].numpy(), len(b[3]) - 1) for b in batches]
        assert raw_view(bus.view(t_raw, 0, records[0].publish(bus, t_raw)))[0].is_pinned(), \
            "raw-batch records must be pinned: the H2D reads them in place"
        pub = OutboundPublisher(bus, t_out, eng.lib, eng.out_cap, rank=rank, world=world)
        runner = PipelinedRunner(eng, max_raw_bytes=max_raw, deliver_outbound=not args.no_outbound,
                                 out_target=pub.target, on_outbound=pub.publish)
        cursor = {"next": bus.end_offset(t_raw, 0)}
        inflight = deque()
        bus_stats = {"bus": bus, "pub": pub, "t_raw": t_raw, "group": group, "cursor": cursor}

        def run(k):
            records[k % len(records)].publish(bus, t_raw, 0, ts=now0 + k)     # producer: batch k arrives
            off = cursor["next"]
            cursor["next"] = off + 1
            payload, lens, n, pb = raw_view(bus.view(t_raw, 0, off))           # consumer: read in place
            slot = runner.k % runner.nbuf
            pub.now_ms = now0 + k
            runner.submit(payload, None, n, now_ms=now0 + k, presence=True, lens_host=lens, raw_bytes=pb)
            inflight.append((off, runner.ev_h2d[slot]))
            while inflight and inflight[0][1].query():
                inflight.popleft()
            bus.hold(t_raw, 0, inflight[0][0] if inflight else None)          # in-flight H2D sources stay
            if off >= 2:
                bus.commit(group, t_raw, 0, off - 1)     # batches < off-1: processed and rows published

        def finish():
            runner.flush()
            bus.hold(t_raw, 0, None)
            bus.commit(group, t_raw, 0, cursor["next"])
    elif use_gpu:
        runner = PipelinedRunner(eng, max_raw_bytes=max_raw, deliver_outbound=not args.no_outbound)

        def run(k):
            rh, oh, r, o, lh = batches[k % len(batches)]
            if lh is not None:
                runner.submit(rh, None, len(o) - 1, now_ms=now0 + k, presence=True, lens_host=lh,
                              raw_bytes=int(o[-1]))
            else:
                runner.submit(rh, oh, len(o) - 1, now_ms=now0 + k, presence=True)

        def finish():
            runner.flush()
    else:
        def run(k):
            _, _, r, o, _ = batches[k % len(batches)]
            eng.step(r, o, now0 + k, presence=True)

        def finish():
            pass

    for k in range(args.warmup):
        run(k)
    finish()
    barrier()
    s0 = eng.stats_dict()
    barrier()
    t_start = time.perf_counter()
    for k in range(args.warmup, args.warmup + args.steps):
        run(k)
    finish()
    barrier()
    elapsed = time.perf_counter() - t_start
    s1 = eng.stats_dict()
    ev = s1["events"] - s0["events"]
    persisted = s1["persisted"] - s0["persisted"]
    msgs = s1["messages"] - s0["messages"]
    rule_alerts = s1["rule_alerts"] - s0["rule_alerts"]
    # whole-job aggregate: max time over ranks, sum of events
    if world > 1:
        t = torch.tensor([elapsed, ev, persisted, msgs, rule_alerts], dtype=torch.float64,
                         device=torch.device("cuda", local) if use_gpu else "cpu")
        tmax = t[:1].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        elapsed = float(tmax.item())
        ev, persisted, msgs, rule_alerts = (int(x) for x in t[1:].tolist())
    value = ev / elapsed
    if rank == 0:
        out = {
            "metric": "device_events_per_sec",
            "value": round(value, 1),
            "unit": "events/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp64/int64 (event values as in the reference; no reduced precision)",
            "data": "synthetic: protobuf device payloads (reference sitewhere.proto) from a random-token fleet",
            "config": {
                "model": "sitewhere-inbound-pipeline",
                "stages": "decode>rekey>validate>dedup>persist+enrich>device-state>zone-rules>presence>outbound",
                "global_batch": args.msgs * world,
                "seq_len": 1,
                "parallelism": f"dp{world} (device-sharded, all-to-all re-key)",
                "payloads_per_gpu_step": args.msgs,
                "devices_per_gpu": args.devices,
                "tenants": 1,
                "zones": args.zones,
                "engine": args.engine,
                "cpu_threads": getattr(eng, "threads", None),
                "framing": args.framing,
                "bus": bool(bus_stats),
            },
            "detail": {
                "events": ev, "persisted": persisted, "payloads": msgs, "rule_alerts": rule_alerts,
                "persisted_per_sec": round(persisted / elapsed, 1),
                "payload_bytes_per_gpu_step": int(max_raw), "setup_s": round(setup_s, 1),
                "h2d_bytes_per_gpu_step": int(max_raw) + int(max(
                    (b[4].numel() if b[4] is not None else 4 * len(b[3])) for b in batches)),
                "registered_devices_rank0": n_dev,
                **({"bus": {"raw_topic_records": bus_stats["bus"].end_offset(bus_stats["t_raw"], 0),
                            "raw_committed": bus_stats["bus"].committed(bus_stats["group"], bus_stats["t_raw"], 0),
                            "enriched_batches_published": bus_stats["pub"].published,
                            "enriched_rows_published": bus_stats["pub"].rows,
                            "enriched_buffers": bus_stats["pub"].n_alloc}} if bus_stats else {}),
            },
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
