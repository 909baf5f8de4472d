#!/usr/bin/env python3
"""Headline benchmark: device events/sec through the SiteWhere inbound pipeline to durable storage.

Reference headline (BASELINE.json): "device events/sec through the Kafka pipeline" --
decode -> inbound validation -> event persistence -> enrichment -> consumers
(device state, rule processing, outbound connectors).  The reference publishes no
number, so ``vs_baseline`` is null.

One step = one micro-batch of ``--msgs`` protobuf device payloads per GPU, run end to end:
  raw batch produced to the raw-payload topic of the native commit log (zero-copy, pinned record)
  -> consumed in place -> H2D of the raw wire bytes straight from the topic -> GPU decode -> [N>1:
  owner partition + RCCL all-to-all re-keying by device token, the analogue of Kafka key
  partitioning] -> registry lookup + assignment validation -> alternate-id dedup -> persist into
  the HBM event store with enrichment -> device-state merge -> zone-test rules (point-in-polygon,
  generated alerts persisted too) -> presence scan -> durable block encoded on the GPU
  (``k_seg_encode``) -> copy-engine D2H of the compressed block -> fdatasync'd segment file
  (O_DIRECT, group commit) + the same block published in place to the enriched-batch topic ->
  rejected messages (unregistered devices, registrations, acks) routed per payload to their topics
  -> raw offsets committed once their block is durable.  The timed region ends when every block
  of the timed steps is on disk.
The fleet is the realistic mix: every event carries an alternate id (dedup active), ~0.5% of the
payloads come from unregistered devices, and registrations / acknowledgements are mixed in.
Weak scaling: per-GPU payloads and per-GPU device shard are fixed as N grows.

Launch: ``python bench.py --gpus 1 --steps 200 --warmup 20`` or under torch.distributed.run
for N > 1 (one rank per GPU, RCCL).
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np


def parse():
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)   # ~0.3 s timed at N=1: steady state, not warm-up
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--msgs", type=int, default=1 << 20, help="payloads per GPU per step")
    ap.add_argument("--devices", type=int, default=1 << 20, help="registered devices per GPU")
    ap.add_argument("--mx-per-msg", type=int, default=1)
    ap.add_argument("--batches", type=int, default=6, help="distinct pre-generated batches to cycle")
    ap.add_argument("--zones", type=int, default=16)
    ap.add_argument("--store", type=int, default=1 << 27, help="HBM event-store capacity per GPU (events)")
    ap.add_argument("--engine", choices=["gpu", "cpu", "oracle"], default="gpu",
                    help="gpu: MI355X kernels; cpu: native multi-threaded C++ engine; oracle: Python reference")
    ap.add_argument("--framing", choices=["varint", "offsets"], default="varint",
                    help="raw-batch framing on the wire to the GPU (varint lengths or u32 offsets)")
    ap.add_argument("--alt-ids", action=argparse.BooleanOptionalAction, default=True,
                    help="every event carries an alternate id (dedup active)")
    ap.add_argument("--p-unregistered", type=float, default=0.005)
    ap.add_argument("--p-register", type=float, default=0.0005)
    ap.add_argument("--p-ack", type=float, default=0.0005)
    ap.add_argument("--dedup-filter-ids", type=int, default=(1 << 29) - (1 << 22),
                    help="store-backed alternate-id filter: ids per generation (4 generations; 0 = off)")
    ap.add_argument("--seed-filter-batches", type=int, default=0,
                    help="(rehearsal) seed every rank's store-backed filter with the alternate ids of the first K "
                         "pre-generated batches of every rank, never stored: filter false positives on demand, "
                         "which their owners settle (pipeline/recheck.py).  Host engines only (the GPU path "
                         "stamps fresh ids into every batch)")
    ap.add_argument("--p-meta", type=float, default=0.1,
                    help="share of events carrying metadata entries (stored with the event, like the reference)")
    ap.add_argument("--durable", action=argparse.BooleanOptionalAction, default=True,
                    help="persist every step's events to fdatasync'd segment files (the headline)")
    ap.add_argument("--durable-dir", default=os.environ.get("SW_DURABLE_DIR"),
                    help="segment directory, or a comma-separated list (one per disk): local rank r writes to "
                         "dirs[r %% len(dirs)] (default: a fresh directory under the temp dir, removed at exit)")
    ap.add_argument("--disk-probe-mb", type=int, default=int(os.environ.get("SW_DISK_PROBE_MB", 256)),
                    help="before timing, every rank writes this much with O_DIRECT + fdatasync to its segment "
                         "directory at the same time: the node's aggregate disk bandwidth (0 = skip)")
    ap.add_argument("--durable-retention-gb", type=float, default=48.0,
                    help="oldest segment files beyond this are deleted (bounded disk use); 0 = keep all")
    ap.add_argument("--direct-io", action=argparse.BooleanOptionalAction, default=True)
    ap.add_argument("--read-threads", type=int, default=0,
                    help="reader threads querying the durable store during the timed steps (list by assignment "
                         "/ area, by id, by alternate id: persistence/read_load.py); 0 = ingest only")
    ap.add_argument("--read-pause-ms", type=float, default=0.0, help="pause between one reader's queries")
    ap.add_argument("--n-customers", type=int, default=97, help="customers of the fleet (assignment i: i %% n)")
    ap.add_argument("--n-areas", type=int, default=31, help="areas of the fleet (assignment i: i %% n)")
    ap.add_argument("--n-assets", type=int, default=1009, help="assets of the fleet (assignment i: i %% n; 0 = "
                                                              "one asset per device)")
    ap.add_argument("--no-outbound", action="store_true", help="(diagnostic) skip the D2H outbound copy")
    ap.add_argument("--bus", action=argparse.BooleanOptionalAction, default=True,
                    help="GPU engine: consume raw batches from, and publish enriched batches to, commit-log "
                         "topics in place (pipeline/bus_io.py); --no-bus feeds pinned batches directly")
    return ap.parse_args()


def durable_dirs(args) -> list[str]:
    return [d for d in (args.durable_dir or "").split(",") if d]


def open_durable(args, rank, dev):
    """(directory to remove at exit or None, DurableEventStore, boot id) of this rank's segments.
    With several ``--durable-dir`` entries (one per disk) local rank r uses entry r mod n."""
    from sitewhere_amd.persistence.segments import DurableEventStore
    dirs = durable_dirs(args)
    local_rank = int(os.environ.get("LOCAL_RANK", rank))
    base = dirs[local_rank % len(dirs)] if dirs else None
    tmpdir = base or tempfile.mkdtemp(prefix=f"sw-bench-durable-r{rank}-")
    seg_dir = os.path.join(tmpdir, f"rank{rank}") if base else tmpdir
    if os.path.exists(seg_dir) and base:
        shutil.rmtree(seg_dir)
    retention = int(args.durable_retention_gb * (1 << 30))
    if retention:
        # the ranks sharing a directory share its disk: each keeps at most half its free space / sharers
        local = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1")))
        sharers = max(1, -(-local // max(1, len(dirs)))) if dirs else local
        probe = os.path.abspath(tmpdir)
        while not os.path.exists(probe):
            probe = os.path.dirname(probe)
        free = shutil.disk_usage(probe).free
        retention = max(2 << 30, min(retention, free // (2 * sharers)))
    # the store is indexed in the timed region: every block carries its index trailer, built on the
    # MI355X in the step that encodes it (alternate ids, assignment zone maps, customer / area / asset
    # key tables; csrc/include/swindex.h) and written with the block in the same group commit
    store = DurableEventStore(seg_dir, rank=rank, rotate_bytes=1 << 30, retention_bytes=retention,
                              direct=args.direct_io)
    boot = int(time.time() * 1000)
    # the whole fleet's dictionary (assignment, device, customer, area, asset tokens; context ids): the
    # store's events are resolvable by token, and the readers look up every assignment / context
    from sitewhere_amd.persistence.read_load import bench_dictionary
    asg, ctx = bench_dictionary(int(np.max(dev)) + 1, args.n_customers, args.n_areas, args.n_assets)
    store.add_dictionary(boot, asg=asg, ctx=ctx)
    return (None if base else tmpdir), store, boot


def disk_probe(directory: str, mb: int, direct: bool = True) -> float:
    """Write ``mb`` MiB in 4 MiB O_DIRECT writes (page-aligned buffer) to a scratch file in
    ``directory``, fdatasync, remove it; returns GB/s.  Run by every rank at once (between barriers),
    so the sum over a node's ranks is the node's aggregate bandwidth to its segment directories."""
    import mmap
    os.makedirs(directory, exist_ok=True)
    path = os.path.join(directory, f".disk-probe-{os.getpid()}")
    chunk = 4 << 20
    buf = mmap.mmap(-1, chunk)
    buf.write(os.urandom(4096) * (chunk // 4096))
    flags = os.O_WRONLY | os.O_CREAT | os.O_TRUNC
    if direct and hasattr(os, "O_DIRECT"):
        flags |= os.O_DIRECT
    try:
        try:
            fd = os.open(path, flags, 0o600)
        except OSError:                      # a file system without O_DIRECT: buffered + fdatasync
            fd = os.open(path, flags & ~getattr(os, "O_DIRECT", 0), 0o600)
        t0 = time.perf_counter()
        for _ in range(max(1, mb // 4)):
            os.write(fd, buf)
        os.fdatasync(fd)
        dt = time.perf_counter() - t0
        os.close(fd)
    finally:
        buf.close()
        try:
            os.remove(path)
        except OSError:
            pass
    return (max(1, mb // 4) * chunk) / dt / 1e9


class _HostSink:
    """Block accounting of the host-engine path (same fields as DurableBlockSink)."""

    def __init__(self, store, eng=None):
        self.store = store
        self.eng = eng
        self.bytes = self.rows = self.blocks = self.index_bytes = 0

    def add(self, blk):
        if self.eng is not None:
            # the same index trailer the MI355X builds in its step (csrc/native/swindex.cpp here):
            # alternate ids, assignment zone maps, customer / area / asset key tables
            from sitewhere_amd.persistence.segments import index_block
            e = self.eng
            n = e.n_assignments
            ctx = np.stack([e.asg_device[:n], e.asg_customer[:n], e.asg_area[:n], e.asg_asset[:n]], axis=1)
            n0 = len(blk)
            blk = index_block(blk, ctx)
            self.index_bytes += len(blk) - n0
        self.store.add_encoded(blk)
        self.bytes += len(blk)
        self.rows += int(blk[8:12].view(np.uint32)[0])
        self.blocks += 1

    def flush(self):
        self.store.flush()


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
    numa_node = None
    if use_gpu and os.environ.get("SW_NUMA_BIND", "1") != "0":
        # host threads and pinned buffers next to this GPU's PCIe root (before anything is allocated)
        from sitewhere_amd.utils.numa import bind_to_gpu_node
        numa_node = bind_to_gpu_node(local)
    from sitewhere_amd.pipeline.config import EngineConfig
    from sitewhere_amd.pipeline.fleet import FleetSpec, gen_payloads, gen_tokens, fingerprints
    from sitewhere_amd.pipeline.framing import varint_lengths

    n_total_dev = args.devices * world
    spec = FleetSpec(prefix="dev-", n_devices=n_total_dev, p_location=0.25, p_alert=0.05,
                     p_unregistered=args.p_unregistered, mx_per_msg=args.mx_per_msg, n_names=16,
                     with_alternate_id=args.alt_ids, lat0=33.0, lon0=-85.0, span_deg=2.0,
                     p_register=args.p_register, p_ack=args.p_ack, p_meta=args.p_meta,
                     # ranks share the per-step id epoch and keep their ids apart in the counter part
                     # ("<epoch>-<rank:2 hex><message:6 hex>"): a block that mixes ranks' events still
                     # shares the id prefix, so its pages keep the compact hex id mode
                     alt_base=rank << 24)
    assert args.msgs <= 1 << 24, "alternate-id counters hold 2^24 messages per rank and step"
    cfg = EngineConfig(max_msgs=args.msgs, rec_cap=args.msgs * args.mx_per_msg + 4096,
                       gen_cap=max(1 << 16, args.msgs // 2), max_devices=int(n_total_dev * 1.1) + 1024,
                       max_assignments=int(n_total_dev * 1.1) + 1024, store_cap=args.store,
                       # alternate-id window: 2^24 slots = the last ~8M distinct ids per GPU
                       dedup_slots=1 << 24, name_slots=1 << 12, rank=rank, world=world,
                       # store-backed dedup beyond the window (pipeline/dedup_filter.py): 4 generations of
                       # ~2^29 ids = 16 GB of the 288 GB of HBM; the filter always holds the newest ~1.6B
                       # ids and the durable store is bounded to that many rows (retention by rows, set
                       # below), so every stored id stays checked however long the run.  Rechecks are counted.
                       dedup_filter_ids=args.dedup_filter_ids, dedup_filter_gens=4,
                       # (assignment, name) state map: 16 measurement names + 4 alert types + zone alerts per device
                       state_slots=2 * (16 + 4 + args.zones) * int(args.devices * 1.1),
                       presence_missing_ms=8 * 3600 * 1000,
                       # 4 staging slots: the runner drains two steps behind (SW_PIPELINE_DEPTH) and the
                       # reject router gets two step periods per batch
                       extra={"out_buffers": int(os.environ.get("SW_OUT_BUFFERS", 4))})
    if use_gpu:
        from sitewhere_amd.pipeline.gpu_engine import GpuInboundEngine, PipelinedRunner
        eng = GpuInboundEngine(cfg, device=torch.device("cuda", local), group=None)
    elif args.engine == "cpu":
        from sitewhere_amd.pipeline.native_engine import NativeCpuEngine
        eng = NativeCpuEngine(cfg)
    else:
        from sitewhere_amd.pipeline.cpu_engine import CpuInboundEngine
        eng = CpuInboundEngine(cfg)

    # ---- registry: replicated on every rank (the decoding rank sends a record of a registered,
    # assigned device to its owner, fp_hi >> 32 mod world, and rejects the rest itself, where the
    # payload bytes are); the owner keeps the device's state, dedup window and events
    t0 = time.time()
    heap, offs = gen_tokens("dev-", 0, n_total_dev)
    lo, hi = fingerprints(heap, offs)
    dev = eng.register_devices(lo, hi)
    n_dev = int(shard_mask(hi, world, rank).sum())
    eng.set_assignments(dev, dev, customer=dev % args.n_customers, area=dev % args.n_areas,
                        asset=dev % args.n_assets if args.n_assets else dev)
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
    if args.seed_filter_batches and not use_gpu:
        from sitewhere_amd.pipeline.fleet import cpu_decode
        mine = np.concatenate([cpu_decode(b[2], b[3], now0)["alt_hash"] for b in batches[:args.seed_filter_batches]])
        every = [mine]
        if world > 1:
            every = [None] * world
            dist.all_gather_object(every, mine)
        ids = np.concatenate(every)
        eng.filter_seed_begin()
        eng.filter_seed(ids[ids != 0])
    setup_s = time.time() - t0
    max_raw = max(int(b[2].size) for b in batches)

    def barrier():
        if world > 1:
            dist.barrier()
        if use_gpu:
            torch.cuda.synchronize()

    bus_stats = None
    dur = None
    # lossless multi-GPU re-keying: while this rank's carry of spilled records is high, its next
    # round is exchange-only (EngineBase.should_stall) -- the input slows down, nothing is dropped
    stalls = {"rounds": 0}

    def stall(runner) -> bool:
        if world > 1 and getattr(runner, "rounds", False) and eng.should_stall():
            stalls["rounds"] += 1
            runner.submit(None, None, 0, now_ms=now0)
            return True
        return False

    # Several ranks: store-backed dedup rechecks are settled by their owner as a deployment does
    # (pipeline/recheck.py): ids its durable store holds are duplicates, the filter's false
    # positives re-enter the re-key carry (the GPU path re-injects them between rounds, on this
    # thread).  ``held_hashes`` asks the store's alternate-id index; without a store nothing is held.
    from sitewhere_amd.pipeline import recheck
    settled = {"rechecks": 0, "duplicates": 0, "injected": 0, "lost": 0}
    settle_q = []

    def held_hashes(h):
        if dur is None or not len(h):
            return [False] * len(h)
        found = dur["store"].find_alternate_hashes([int(x) for x in h])
        return [int(x) in found for x in h]

    def inject_settled():
        while settle_q:
            try:
                eng.inject_settled(*settle_q[0])
            except RuntimeError as e:               # carry full: retried after the next round drains it
                if "carry full" not in str(e):
                    raise
                return
            settle_q.pop(0)
    tmpdir = None
    boot = 0
    if use_gpu and args.bus and args.framing == "varint":
        # Through the bus: each step the producer side hands raw batch k to the raw-payload topic
        # (zero-copy: the record is the pinned buffer), the engine's consumer reads it in place and
        # DMAs it to HBM.  The step's persisted events are encoded on the GPU into one durable block,
        # the copy engine moves the compressed block to a pinned buffer that is written to the
        # segment store (O_DIRECT + fdatasync) and published in place to the enriched-batch topic.
        # Rejected messages are routed per payload while their raw record is still held.  Raw
        # offsets are committed once the batch's block is durable.
        from collections import deque

        from sitewhere_amd.bus.log import EventBus
        from sitewhere_amd.bus.naming import TopicNaming
        from sitewhere_amd.persistence.segments import DurableBlockSink, DurableEventStore
        from sitewhere_amd.pipeline import routing
        from sitewhere_amd.pipeline.bus_io import OutboundPublisher, RawBatchRecord, raw_view
        bus = EventBus(None, default_partitions=1)
        naming = TopicNaming("sitewhere", f"bench-rank{rank}")
        prefix = naming.tenant_prefix("default")
        t_raw, t_out = prefix + "event-source-raw-payloads", prefix + "inbound-enriched-batches"
        group = prefix + "inbound-processing.raw-payload-consumers"
        route_topics = (naming.unregistered_device_events("default"), naming.device_registration_events("default"),
                        naming.decoded_events("default"), naming.failed_decode_events("default"))
        for t in route_topics:
            bus.topic(t, 8)
            bus.set_retention(t, 64 << 20)
        route_parts = [bus.partitions(t) for t in route_topics]
        bus.topic(t_raw, 1)
        bus.set_retention(t_raw, 16 * max_raw)
        records = [RawBatchRecord(b[2][:int(b[3][-1])], b[4].numpy(), len(b[3]) - 1) for b in batches]
        assert raw_view(bus.view(t_raw, 0, records[0].publish(bus, t_raw)))[0].is_pinned(), \
            "raw-batch records must be pinned: the H2D reads them in place"
        routed = {"records": 0, "payloads": 0, "by_kind": [0, 0, 0, 0], "control_decoded": 0}

        def on_rejects(off, refs, compact):
            # the GPU copied the rejected payloads into `compact`; the router parses only those and
            # writes the reference's Kafka payloads natively (the held record serves overflow refs)
            if world > 1:
                # rechecks came as packages (record + strings): their owner settles them by
                # alternate id against its store; false positives re-enter the carry between rounds
                recs, spans, heap, lost = recheck.unpack_rechecks(refs, compact)
                if len(recs) or lost:
                    c = recheck.settle(eng, recs, spans, heap, held_hashes, by_hash=True,
                                       inject=lambda *x: settle_q.append(x))
                    for key in ("rechecks", "duplicates", "injected"):
                        settled[key] += c[key]
                    settled["lost"] += lost
            t0 = time.perf_counter()
            payload = raw_view(bus.view(t_raw, 0, off))[0]
            rr = routing.route_refs(compact, refs, rank, "bench", route_parts, raw=payload.data_ptr())
            t1 = time.perf_counter()
            routed["payloads"] += rr.payloads
            per = bus.append_routed(route_topics, rr)
            routed["records"] += sum(per)
            for kind, c in enumerate(per):
                routed["by_kind"][kind] += c
            routed["route_s"] = routed.get("route_s", 0.0) + (t1 - t0)
            routed["publish_s"] = routed.get("publish_s", 0.0) + (time.perf_counter() - t1)
            routed["jobs"] = routed.get("jobs", 0) + 1

        if args.durable:
            tmpdir, store, boot = open_durable(args, rank, dev)
            # the store keeps no row whose id the filter has forgotten (the blocks in flight are the
            # slack; EngineConfig.filter_retention_rows accounts for the file being written)
            store.limit_retention_rows(cfg.filter_retention_rows(16 * cfg.rec_cap))
            sink = DurableBlockSink(store, eng.lib, boot, rank=rank, world=world, bus=bus, topic=t_out)
            bus.set_retention(t_out, 64 << 20)
            dur = {"store": store, "sink": sink}
            runner = PipelinedRunner(eng, max_raw_bytes=max_raw, deliver_outbound=False, block_sink=sink, nbuf=4,
                                     on_rejects=on_rejects)
        else:
            pub = OutboundPublisher(bus, t_out, eng.lib, eng.out_cap, rank=rank, world=world)
            runner = PipelinedRunner(eng, max_raw_bytes=max_raw, deliver_outbound=not args.no_outbound,
                                     out_target=pub.target, on_outbound=pub.publish, on_rejects=on_rejects)
        # The synthetic producer: every event carries a fresh alternate id (the replayed batches get a
        # new id epoch stamped in place, natively, one step ahead on a producer thread) -- otherwise
        # dedup would rightly discard every replayed event.
        from concurrent.futures import ThreadPoolExecutor

        from sitewhere_amd.pipeline.bus_io import VALUE_HDR
        from sitewhere_amd.pipeline.fleet import alt_positions, stamp_positions
        # the producer stamps batch k+AHEAD while k is published: two stamps in flight, each on
        # several threads, so generating fresh ids never paces the pipeline; a batch is re-stamped
        # only once every step that read its record (H2D, compute, reject routing) is long done
        AHEAD = 2
        assert not args.alt_ids or len(batches) >= AHEAD + 4, "the producer lookahead needs >= 6 distinct batches"
        producer = ThreadPoolExecutor(AHEAD, thread_name_prefix="producer") if args.alt_ids else None
        stamps = {}
        # where each batch's alternate-id epochs sit, found once: stamping then only writes
        alt_pos = [alt_positions(rec.ptr + VALUE_HDR, b[3]) for rec, b in zip(records, batches)] \
            if args.alt_ids else None

        def stamp(k):
            rec = records[k % len(records)]
            return stamp_positions(rec.ptr + VALUE_HDR, alt_pos[k % len(records)],
                                   (0x5717 << 48) | k, threads=int(os.environ.get("SW_STAMP_THREADS", 8)))

        if producer is not None:
            for j in range(AHEAD):
                stamps[j] = producer.submit(stamp, j)
        cursor = {"next": bus.end_offset(t_raw, 0), "committed": bus.end_offset(t_raw, 0)}
        inflight = deque()
        bus_stats = {"bus": bus, "t_raw": t_raw, "group": group, "cursor": cursor, "routed": routed,
                     "route_topics": route_topics}

        def commit_durable():
            if dur is None:
                return
            done = dur["sink"].committable()
            if done:
                cursor["durable"] = max(cursor.get("durable", 0), max(o for o in done if o is not None) + 1)
            # commit what is durable AND whose rejects are routed (the router runs on its own thread)
            floor = runner.rejects_floor()
            upto = cursor.get("durable", cursor["committed"]) if floor is None else min(cursor.get("durable", 0), floor)
            if upto > cursor["committed"]:
                cursor["committed"] = upto
                bus.commit(group, t_raw, 0, upto)

        def run(k):
            inject_settled()
            if stall(runner):
                commit_durable()
                return
            if producer is not None:
                stamps.pop(k).result()                        # batch k's fresh alternate ids
            records[k % len(records)].publish(bus, t_raw, 0, ts=now0 + k)     # producer: batch k arrives
            if producer is not None:
                stamps[k + AHEAD] = producer.submit(stamp, k + AHEAD)
            off = cursor["next"]
            cursor["next"] = off + 1
            # the consumer holds every record not yet committed: H2D in flight, rejects to route,
            # block not yet durable
            bus.hold(t_raw, 0, cursor["committed"] if dur is not None else off)
            payload, lens, n, pb = raw_view(bus.view(t_raw, 0, off))           # consumer: read in place
            slot = runner.k % runner.nbuf
            runner.submit(payload, None, n, now_ms=now0 + k, presence=True, lens_host=lens, raw_bytes=pb, tag=off)
            if dur is None:
                inflight.append((off, runner.ev_h2d[slot]))
                while inflight and inflight[0][1].query():
                    inflight.popleft()
                bus.hold(t_raw, 0, inflight[0][0] if inflight else None)
                if off >= 2:
                    bus.commit(group, t_raw, 0, off - 1)     # batches < off-1: processed and rows published
            else:
                commit_durable()

        def finish():
            runner.flush()
            inject_settled()                                  # settled after the last round: carried
            if dur is not None:
                dur["sink"].flush()                           # every block of the run is on disk
                commit_durable()
            bus.hold(t_raw, 0, None)
            if dur is None:
                bus.commit(group, t_raw, 0, cursor["next"])
    elif use_gpu:
        runner = PipelinedRunner(eng, max_raw_bytes=max_raw, deliver_outbound=not args.no_outbound)

        def run(k):
            if stall(runner):
                return
            rh, oh, r, o, lh = batches[k % len(batches)]
            if lh is not None:
                runner.submit(rh, None, len(o) - 1, now_ms=now0 + k, presence=True, lens_host=lh,
                              raw_bytes=int(o[-1]))
            else:
                runner.submit(rh, oh, len(o) - 1, now_ms=now0 + k, presence=True)

        def finish():
            runner.flush()
    else:
        if args.durable:        # host engines encode the same blocks on the CPU (swseg_encode)
            tmpdir, store, boot = open_durable(args, rank, dev)
            # the store keeps no row whose id the filter has forgotten (the blocks in flight are the
            # slack; EngineConfig.filter_retention_rows accounts for the file being written)
            store.limit_retention_rows(cfg.filter_retention_rows(16 * cfg.rec_cap))
            dur = {"store": store, "sink": _HostSink(store, eng)}

        def run(k):
            _, _, r, o, _ = batches[k % len(batches)]
            if eng.should_stall():                  # skewed keys: an exchange-only round instead
                stalls["rounds"] += 1
                r, o = np.zeros(64, np.uint8), np.zeros(1, np.uint32)
            res = eng.step(r, o, now0 + k, presence=True)
            if dur is not None:
                dur["sink"].add(eng.encode_block(now0 + k, res, boot=boot))
            if world > 1:                           # the owner settles its rechecks (pipeline/recheck.py)
                for key, v in recheck.settle_rechecks(eng, res, held_hashes, by_hash=True).items():
                    settled[key] += v

        def finish():
            if dur is not None:
                dur["sink"].flush()

    probe = None
    if dur is not None and args.disk_probe_mb > 0:
        # every rank at once, between barriers: per-rank and node-aggregate O_DIRECT write bandwidth
        barrier()
        gbps = disk_probe(dur["store"].dir, args.disk_probe_mb, args.direct_io)
        agg = gbps
        if world > 1:
            tg = torch.tensor([gbps], dtype=torch.float64, device=torch.device("cuda", local) if use_gpu else "cpu")
            dist.all_reduce(tg, op=dist.ReduceOp.SUM)
            agg = float(tg.item())
        probe = {"mb_per_rank": args.disk_probe_mb, "rank0_gbps": round(gbps, 2), "node_gbps": round(agg, 2),
                 "dirs": max(1, len(durable_dirs(args)))}
    for k in range(args.warmup):
        run(k)
    finish()
    barrier()
    s0 = eng.stats_dict()
    settled0 = dict(settled)
    d0 = dur["store"].seg.stats() if dur else None
    sk0 = (dur["sink"].bytes, dur["sink"].rows, dur["sink"].blocks, getattr(dur["sink"], "disk_wait_s", 0.0),
           getattr(dur["sink"], "index_bytes", 0)) if dur else None
    r0 = dict(bus_stats["routed"], by_kind=list(bus_stats["routed"]["by_kind"])) if bus_stats else None
    reads = None
    if dur is not None and args.read_threads > 0:
        from sitewhere_amd.persistence.read_load import ReadLoad
        # the readers' Python holds the interpreter between their native calls: hand it back to
        # the step loop every 0.2 ms rather than the default 5 ms
        sys.setswitchinterval(2e-4)
        reads = ReadLoad(dur["store"], int(np.max(dev)) + 1, threads=args.read_threads,
                         pause_s=args.read_pause_ms / 1e3, seed=rank, n_area=args.n_areas,
                         n_cust=args.n_customers, n_asset=args.n_assets or int(np.max(dev)) + 1)
    # the setup's long-lived objects (registry, dictionaries: millions with --read-threads) leave the
    # collector's view: a full collection over them would stall every thread of the process
    import gc
    gc.collect()
    gc.freeze()
    barrier()
    if reads is not None:
        reads.start()
    t_start = time.perf_counter()
    t_steps = []
    for k in range(args.warmup, args.warmup + args.steps):
        run(k)
        t_steps.append(time.perf_counter())
    finish()
    t_fin = time.perf_counter()
    read_stats = reads.stop() if reads is not None else None
    barrier()
    elapsed = time.perf_counter() - t_start
    # where the timed region went (rank 0's clock): submit intervals of the steps, then the drain
    # (the steps still in flight, their blocks made durable)
    step_ms = np.diff(np.asarray([t_start] + t_steps)) * 1e3
    timeline = {"submit_ms_p50": round(float(np.median(step_ms)), 3), "submit_ms_max": round(float(step_ms.max()), 3),
                "submit_ms_first3": [round(float(x), 3) for x in step_ms[:3]],
                "drain_ms": round((t_fin - t_steps[-1]) * 1e3, 3)} if len(step_ms) else None
    s1 = eng.stats_dict()
    ev = s1["events"] - s0["events"]
    persisted = s1["persisted"] - s0["persisted"]
    msgs = s1["messages"] - s0["messages"]
    rule_alerts = s1["rule_alerts"] - s0["rule_alerts"]
    rank_elapsed = elapsed
    # whole-job aggregate: max time over ranks, sum of events
    per_rank = None
    if world > 1:
        dev_t = torch.device("cuda", local) if use_gpu else "cpu"
        t = torch.tensor([elapsed, ev, persisted, msgs, rule_alerts], dtype=torch.float64, device=dev_t)
        tmax = t[:1].clone()
        gathered = [torch.zeros(1, dtype=torch.float64, device=dev_t) for _ in range(world)]
        dist.all_gather(gathered, t[:1].clone())
        per_rank = [round(float(x.item()), 6) for x in gathered]
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        elapsed = float(tmax.item())
        ev, persisted, msgs, rule_alerts = (int(x) for x in t[1:].tolist())
    value = ev / elapsed
    # ---- conservation: every decoded event is persisted or rejected (and every reject routed),
    # every persisted row is in a durable block, every raw record committed -- summed over ranks
    from sitewhere_amd.models.columnar import STAT_NAMES
    cons = [s1[k] - s0[k] for k in STAT_NAMES]
    cons.append(dur["sink"].rows - sk0[1] if dur else -1)
    cons.append(bus_stats["routed"]["payloads"] - r0["payloads"] if bus_stats else -1)
    settle_keys = ["settled_" + k for k in settled]
    cons += [settled[k] - settled0[k] for k in settled]
    if world > 1:
        ct = torch.tensor(cons, dtype=torch.int64, device=torch.device("cuda", local) if use_gpu else "cpu")
        dist.all_reduce(ct, op=dist.ReduceOp.SUM)
        cons = [int(x) for x in ct.tolist()]
    c = dict(zip(STAT_NAMES + ["durable_rows", "routed_payloads"] + settle_keys, cons))
    rejected = c["unregistered"] + c["unassigned"] + c["duplicates"] + c["decode_errors"] + c["control"] + \
        c["dedup_rechecks"]
    checks = {"persisted == events - rejected + rule_alerts + presence":
              c["persisted"] == c["events"] - rejected + c["rule_alerts"] + c["presence_events"],
              "no dedup / state / shuffle overflow": c["dedup_overflow"] == 0 and c["state_overflow"] == 0
              and c["shuffle_overflow"] == 0}
    if dur:
        checks["durable rows == persisted"] = c["durable_rows"] == c["persisted"]
        checks["every block durable"] = bool(dur["sink"].store.durable() >= dur["sink"].store.seg.last_token)
    if world > 1 and cfg.str_cap:
        checks["rechecks settled by their owner == duplicates + re-injected"] = \
            c["settled_rechecks"] + c["settled_lost"] == c["dedup_rechecks"] and \
            c["settled_rechecks"] == c["settled_duplicates"] + c["settled_injected"] and c["settled_lost"] == 0
    if bus_stats:
        # one rank routes its rechecks' payloads to the per-event path; several settle them
        routed_rk = c["dedup_rechecks"] if world == 1 or not cfg.str_cap else 0
        checks["routed payloads == unregistered + unassigned + control + decode errors + rechecks"] = \
            c["routed_payloads"] == c["unregistered"] + c["unassigned"] + c["control"] + c["decode_errors"] + \
            routed_rk
        checks["raw topic fully committed"] = \
            bus_stats["bus"].committed(bus_stats["group"], bus_stats["t_raw"], 0) == \
            bus_stats["bus"].end_offset(bus_stats["t_raw"], 0)
    conservation_ok = all(checks.values())
    detail = {
        "events": ev, "persisted": persisted, "payloads": msgs, "rule_alerts": rule_alerts,
        "persisted_per_sec": round(persisted / elapsed, 1),
        "payload_bytes_per_gpu_step": int(max_raw), "setup_s": round(setup_s, 1),
        "h2d_bytes_per_gpu_step": int(max_raw) + int(max(
            (b[4].numel() if b[4] is not None else 4 * len(b[3])) for b in batches)),
        "registered_devices_rank0": int(len(dev)), "owned_devices_rank0": n_dev,
        "rejected_rank0": {k: s1[k] - s0[k] for k in ("unregistered", "unassigned", "duplicates", "decode_errors",
                                                       "control")},
        "numa_node": numa_node,
        "backend": dist.get_backend() if world > 1 else None,
        "world": dist.get_world_size() if world > 1 else 1,
        "rank_elapsed_s": per_rank if per_rank is not None else [round(rank_elapsed, 6)],
        "timeline_rank0": timeline,
        "conservation": {"ok": conservation_ok, "failed": [k for k, v in checks.items() if not v],
                         "checked": len(checks)},
    }
    if world > 1:
        # what one rank sends per step: its record slab for every destination, plus (lossless
        # records) the string refs and string byte slabs beside them
        detail["exchange_bytes_per_rank_step"] = world * cfg.shuf_cap * 64 + \
            (world * cfg.shuf_cap * 16 + world * cfg.str_cap if cfg.str_cap else 0)
        if hasattr(eng, "string_drops"):
            drops = torch.tensor(list(eng.string_drops().values()), dtype=torch.int64,
                                 device=torch.device("cuda", local) if use_gpu else "cpu")
            dist.all_reduce(drops, op=dist.ReduceOp.SUM)
            # lossless re-key: a record whose slab is full waits in the carry with its strings; only
            # a record whose strings alone exceed a whole slab goes without them
            detail["string_exchange"] = {"bytes_per_slot": cfg.str_bytes, "slab_bytes": cfg.str_cap,
                                         "carry_heap_bytes": cfg.carry_str_cap,
                                         "records_without_strings": {k: int(v) for k, v in
                                                                     zip(eng.string_drops(), drops.tolist())}}
        detail["shuffle_deferred"] = s1.get("shuffle_deferred", 0) - s0.get("shuffle_deferred", 0)
        detail["shuffle_overflow"] = s1.get("shuffle_overflow", 0) - s0.get("shuffle_overflow", 0)
        detail["stall_rounds"] = stalls["rounds"]
        detail["rechecks_settled"] = {k: c["settled_" + k] for k in settled}
    if bus_stats:
        r1 = bus_stats["routed"]
        bus = bus_stats["bus"]
        detail["bus"] = {"raw_topic_records": bus.end_offset(bus_stats["t_raw"], 0),
                         "raw_committed": bus.committed(bus_stats["group"], bus_stats["t_raw"], 0),
                         "rejects_routed_records": r1["records"] - r0["records"],
                         "rejects_routed_payloads": r1["payloads"] - r0["payloads"],
                         "routed_by_topic": {t.rsplit(".", 1)[-1]: r1["by_kind"][i] - r0["by_kind"][i]
                                             for i, t in enumerate(bus_stats["route_topics"])}}
        if r1.get("jobs"):
            detail["bus"]["router_ms_per_job"] = {"route": round(1000 * r1["route_s"] / r1["jobs"], 3),
                                                  "publish": round(1000 * r1["publish_s"] / r1["jobs"], 3)}
    if use_gpu and getattr(runner, "trace", None) is not None:
        detail["runner_trace_ms_per_step"] = {k: round(1000 * v / (args.steps + args.warmup), 3)
                                              for k, v in runner.trace.items()}
    if dur:
        d1 = dur["store"].seg.stats()
        sk = dur["sink"]
        nbytes, nrows, nblocks = sk.bytes - sk0[0], sk.rows - sk0[1], sk.blocks - sk0[2]
        detail["durable"] = {
            "blocks": nblocks, "rows": nrows, "block_bytes": nbytes,
            "bytes_per_event": round(nbytes / max(1, nrows), 3),
            # of which the block index trailers (the store's read-side indexes, built in the step)
            "index_bytes_per_event": round((getattr(sk, "index_bytes", 0) - sk0[4]) / max(1, nrows), 3),
            "durable_bytes_per_s": round((d1["bytes_written"] - d0["bytes_written"]) / elapsed, 1),
            "disk_bytes_written": d1["bytes_written"] - d0["bytes_written"],
            # the segment writer's time in the timed region: block writes, fdatasync, waiting for
            # the copier (scan images + trailer copies for reads), and the copier's own time
            "writer_ms": {k: round((d1[k] - d0[k]) / 1e6, 2) for k in ("write_ns", "sync_ns", "copier_wait_ns",
                                                                      "copier_ns")},
            "fdatasyncs": d1["syncs"] - d0["syncs"], "direct_io": bool(d1["direct_io"]),
            "retention_deleted_bytes": d1["deleted_bytes"], "all_durable": sk.store.durable() >= sk.store.seg.last_token,
            # time the pipeline waited for the disk (block buffers all queued, not yet durable):
            # > 0 means this rank's step was storage-bound, e.g. several ranks sharing one disk
            "disk_wait_ms_per_step": round(1000 * (getattr(sk, "disk_wait_s", 0.0) - sk0[3]) / args.steps, 3),
            # what the disks can take: this rank's and the node's (all ranks at once) O_DIRECT bandwidth,
            # vs what the step needs (bytes per step x steps per second, whole job)
            "disk_probe": probe,
            "needed_gbps_job": round(world * (nbytes / max(1, args.steps)) / (elapsed / args.steps) / 1e9, 2),
        }
    if read_stats is not None:
        detail["reads"] = read_stats          # this rank's query latencies while it ingested
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
            "data": "synthetic: protobuf device payloads (reference sitewhere.proto) from a random-token fleet; "
                    f"alternate ids {'on' if args.alt_ids else 'off'}, {args.p_unregistered:.2%} unregistered, "
                    f"{args.p_register:.2%} registrations, {args.p_ack:.2%} acks",
            "config": {
                "model": "sitewhere-inbound-pipeline",
                "stages": "decode>rekey>validate>dedup>persist+enrich>device-state>zone-rules>presence>"
                          + ("gpu-encode>durable-store(fdatasync)>" if dur else "outbound>") + "reject-routing",
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
                "durable": bool(dur),
            },
            "detail": detail,
        }
        print(json.dumps(out), flush=True)
    if dur:
        dur["store"].close()
        if tmpdir:
            shutil.rmtree(tmpdir, ignore_errors=True)
    if world > 1:
        dist.destroy_process_group()
    if not conservation_ok:
        print(f"bench: conservation check failed on rank {rank}: {[k for k, v in checks.items() if not v]} {c}",
              file=sys.stderr, flush=True)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
