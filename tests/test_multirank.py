"""Multi-rank (sharded) pipeline without a cluster.

* loopback: W engine shards in one process exchange their owner slabs by plain copies; the
  GPU shards (gpu-marked) must match the CPU oracle shards record for record.
* gloo: 2 real processes run the CPU engine over torch.distributed all_to_all_single.
Reference analogue: Kafka key partitioning of the decoded-events topic by device token.
"""
import os

import numpy as np
import pytest

from sitewhere_amd.models.columnar import EVENT_REC
from sitewhere_amd.pipeline.config import EngineConfig
from sitewhere_amd.pipeline.cpu_engine import CpuInboundEngine
from sitewhere_amd.pipeline.fleet import fingerprints, gen_tokens

from pipeline_scenarios import NOW, fleet_batch, canon_out, SQUARE
from tests.conftest import gpu_available

W = 3
N_DEV = 900


def shard_fleet(e, world, rank):
    """Every rank registers the whole fleet (the registry is replicated: the decoding rank decides
    whether a record goes to its device's owner or is rejected where its payload is); the owner
    keeps the device's state, dedup window and events.  Returns the devices this rank owns."""
    heap, offs = gen_tokens("dev-", 0, N_DEV)
    lo, hi = fingerprints(heap, offs)
    mine = ((hi >> np.uint64(32)) % np.uint64(world)) == rank
    dev = e.register_devices(lo, hi)
    e.set_assignments(dev, dev, customer=dev % 7, area=dev % 5, asset=dev % 3)
    from sitewhere_amd.pipeline.engine_base import Zone, ZoneTest
    e.set_zone_rules([Zone("z1", SQUARE)], [ZoneTest("z1", "inside", "zone.enter", 2)])
    return int(mine.sum())


def cpu_shards():
    shards = [CpuInboundEngine(EngineConfig.small(world=W, rank=r)) for r in range(W)]
    for r, e in enumerate(shards):
        shard_fleet(e, W, r)
    return shards


def cpu_loopback_step(shards, batches, now):
    decoded = [e.decode_phase(raw, offs, now) for e, (raw, offs) in zip(shards, batches)]
    # with the string exchange on, a slab takes the prefix of records whose strings fit it too
    slabs = [e.partition(recs, spans=e._dec_spans, raw=np.asarray(raw, np.uint8)) if e.cfg.str_cap
             else e.partition(recs) for e, (recs, _), (raw, _) in zip(shards, decoded, batches)]
    out = []
    for q, e in enumerate(shards):
        recv = np.stack([slabs[r][0][q] for r in range(W)])
        rcnt = [slabs[r][1][q] for r in range(W)]
        work = e.unpack(recv, rcnt)
        out.append(e.process_phase(work, len(batches[q][1]) - 1, now, decoded[q][1], presence=False))
    return out


def test_cpu_loopback_conserves_events():
    shards = cpu_shards()
    batches = [fleet_batch(1500, seed=40 + r, n_dev=N_DEV) for r in range(W)]
    res = cpu_loopback_step(shards, batches, NOW)
    total_events = sum(r.n_events for r in res)
    single = CpuInboundEngine(EngineConfig.small(max_msgs=8192))
    shard_fleet(single, 1, 0)
    ref = [single.step(raw, offs, NOW, presence=False) for raw, offs in batches]
    assert total_events == sum(r.n_events for r in ref)
    assert sum(r.n_persisted for r in res) == sum(r.n_persisted for r in ref)
    # every persisted event lands on the owner of its device
    for r, res_r in enumerate(res):
        assert (res_r.event_ids() % W == r).all()


def test_rejects_stay_with_their_payload():
    """Records of unregistered devices are rejected by the rank that decoded them -- its raw batch
    holds the payload the slow path routes -- and every reject ref points into that batch."""
    from sitewhere_amd.models.columnar import ST_UNREGISTERED
    shards = cpu_shards()
    batches = [fleet_batch(1500, seed=60 + r, n_dev=N_DEV) for r in range(W)]
    res = cpu_loopback_step(shards, batches, NOW)
    unreg = 0
    for r, res_r in enumerate(res):
        st = res_r.reject_status
        assert (res_r.rejects["src_rank"] == r).all()          # never a remote record
        unreg += int((st == ST_UNREGISTERED).sum())
    single = CpuInboundEngine(EngineConfig.small(max_msgs=8192))
    shard_fleet(single, 1, 0)
    ref = [single.step(raw, offs, NOW, presence=False) for raw, offs in batches]
    assert unreg == sum(int((x.reject_status == ST_UNREGISTERED).sum()) for x in ref) > 0


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X GPU")
def test_gpu_loopback_matches_cpu_oracle():
    import torch
    from sitewhere_amd.pipeline.gpu_engine import GpuInboundEngine

    g = [GpuInboundEngine(EngineConfig.small(world=W, rank=r)) for r in range(W)]
    for r, e in enumerate(g):
        shard_fleet(e, W, r)
    c = cpu_shards()
    for step in range(3):
        batches = [fleet_batch(1500, seed=70 + 10 * step + r, n_dev=N_DEV) for r in range(W)]
        now = NOW + step * 1000
        # GPU: decode+partition on every shard, loopback exchange by device copies, then process
        devbufs = []
        for e, (raw, offs) in zip(g, batches):
            rd = torch.from_numpy(np.concatenate([raw, np.zeros(64, np.uint8)])).cuda()
            od = torch.from_numpy(offs.view(np.int32)).cuda()
            devbufs.append((rd, od))
            e.prepare(rd, od, len(offs) - 1, now)
            e.phase_decode()
        for q in range(W):
            for r in range(W):
                g[q].recv_slab(r).copy_(g[r].send_slab(q))
                g[q].t["recv_cnt"][r] = g[r].send_count(q)
        for e in g:
            e.phase_process()
        torch.cuda.synchronize()
        gres = [e.collect(e._last_sel, raw) for e, (raw, _) in zip(g, batches)]
        cres = cpu_loopback_step(c, batches, now)
        for r in range(W):
            assert gres[r].n_events == cres[r].n_events
            assert gres[r].n_persisted == cres[r].n_persisted
            assert canon_out(gres[r].out, None) == canon_out(cres[r].out, None)
            assert np.array_equal(gres[r].event_ids(), cres[r].event_ids())
    for r in range(W):
        assert g[r].stats_dict() == c[r].stats_dict()


SPILL = dict(shuffle_slack=0.1, shuffle_pad=0)     # slabs of ~270 records: every step spills


def test_cpu_spill_defers_and_conserves_events():
    """Records beyond a full slab are carried to the next exchange (never dropped): after drain
    steps with empty batches the shards have processed exactly the single-shard event count."""
    shards = [CpuInboundEngine(EngineConfig.small(world=W, rank=r, **SPILL)) for r in range(W)]
    for r, e in enumerate(shards):
        shard_fleet(e, W, r)
    steps = [[fleet_batch(1500, seed=40 + 10 * k + r, n_dev=N_DEV) for r in range(W)] for k in range(3)]
    got = 0
    for k, batches in enumerate(steps):
        got += sum(r.n_events for r in cpu_loopback_step(shards, batches, NOW + k))
    assert sum(int(e.stats[13]) for e in shards) > 0 and sum(len(e.carry) for e in shards) > 0
    empty = (np.zeros(0, np.uint8), np.zeros(1, np.uint32))
    for k in range(20):
        if not any(len(e.carry) for e in shards):
            break
        got += sum(r.n_events for r in cpu_loopback_step(shards, [empty] * W, NOW + 10 + k))
    assert not any(len(e.carry) for e in shards)
    single = CpuInboundEngine(EngineConfig.small(max_msgs=8192))
    shard_fleet(single, 1, 0)
    ref = sum(single.step(raw, offs, NOW, presence=False).n_events for b in steps for raw, offs in b)
    assert got == ref
    assert sum(e.stats_dict()["shuffle_overflow"] for e in shards) == 0


def _gpu_shards(**kw):
    from sitewhere_amd.pipeline.gpu_engine import GpuInboundEngine
    g = [GpuInboundEngine(EngineConfig.small(world=W, rank=r, **kw)) for r in range(W)]
    for r, e in enumerate(g):
        shard_fleet(e, W, r)
    c = [CpuInboundEngine(EngineConfig.small(world=W, rank=r, **kw)) for r in range(W)]
    for r, e in enumerate(c):
        shard_fleet(e, W, r)
    return g, c


def _dev_batch(raw, offs):
    import torch
    return (torch.from_numpy(np.concatenate([raw, np.zeros(64, np.uint8)])).cuda(),
            torch.from_numpy(np.ascontiguousarray(offs, np.uint32).view(np.int32)).cuda())


def _loopback_copy(g):
    for q in range(W):
        for r in range(W):
            g[q].recv_slab(r).copy_(g[r].send_slab(q))
            g[q].t["recv_cnt"][r] = g[r].send_count(q)


def _assert_same(gres, cres):
    for r in range(W):
        assert gres[r].n_events == cres[r].n_events
        assert gres[r].n_persisted == cres[r].n_persisted
        assert canon_out(gres[r].out, None) == canon_out(cres[r].out, None)
        assert np.array_equal(gres[r].event_ids(), cres[r].event_ids())


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X GPU")
def test_gpu_loopback_spill_matches_cpu_oracle():
    """Spilled records (full slabs) are carried in the same deterministic order as the oracle."""
    import torch
    g, c = _gpu_shards(**SPILL)
    empty = (np.zeros(0, np.uint8), np.zeros(1, np.uint32))
    for step in range(5):
        batches = ([fleet_batch(1500, seed=90 + 10 * step + r, n_dev=N_DEV) for r in range(W)] if step < 3
                   else [empty] * W)
        now = NOW + step * 1000
        keep = []
        for e, (raw, offs) in zip(g, batches):
            rd, od = _dev_batch(raw, offs)
            keep.append((rd, od))
            e.prepare(rd, od, len(offs) - 1, now)
            e.phase_decode()
        _loopback_copy(g)
        for e in g:
            e.phase_process()
        torch.cuda.synchronize()
        _assert_same([e.collect(e._last_sel, raw) for e, (raw, _) in zip(g, batches)],
                     cpu_loopback_step(c, batches, now))
    for r in range(W):
        assert g[r].stats_dict() == c[r].stats_dict()
    assert sum(e.stats_dict()["shuffle_deferred"] for e in g) > 0


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X GPU")
def test_gpu_pipelined_rounds_match_serial_oracle():
    """round_async (decode k | process k-1, exchange overlapped) gives each batch exactly the serial
    step's result, one round later; the final round drains the batch in flight."""
    import torch
    g, c = _gpu_shards()
    steps = [[fleet_batch(1500, seed=170 + 10 * k + r, n_dev=N_DEV) for r in range(W)] for k in range(4)]
    cpu = [cpu_loopback_step(c, b, NOW + k * 1000) for k, b in enumerate(steps)]
    keep = []
    for k in range(len(steps) + 1):
        for r, e in enumerate(g):
            if k < len(steps):
                raw, offs = steps[k][r]
                rd, od = _dev_batch(raw, offs)
                keep.append((rd, od))
                done = e.round_async(rd, od, len(offs) - 1, NOW + k * 1000, out_sel=k % 2, exchange=False)
            else:
                done = e.round_async(None, out_sel=k % 2, exchange=False)
            assert done == (k > 0)
        if k < len(steps):
            _loopback_copy(g)
            for e in g:
                e.exchange_done()
        torch.cuda.synchronize()
        if k > 0:
            _assert_same([e.collect(k % 2, None) for e in g], cpu[k - 1])
    assert not any(e.exchange_pending for e in g)
    for r in range(W):
        assert g[r].stats_dict() == c[r].stats_dict()


def _gloo_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    e = CpuInboundEngine(EngineConfig.small(world=world, rank=rank))
    shard_fleet(e, world, rank)
    raw, offs = fleet_batch(1000, seed=500 + rank, n_dev=N_DEV)
    r = e.step(raw, offs, NOW, presence=False)
    keys = _block_string_keys(e.encode_block(NOW, r, boot=5))
    q.put((rank, r.n_events, r.n_persisted, bool((r.event_ids() % world == rank).all()), keys))
    dist.barrier()
    dist.destroy_process_group()


def _block_string_keys(block) -> list:
    """(type, date, value, alternate id, message, metadata) of every row of a durable block."""
    from sitewhere_amd.persistence.segments import decode_block, row_strings
    c = decode_block(block)
    out = []
    for i in range(len(c["etype"])):
        alt, msg, md = row_strings(c, i)
        out.append((int(c["etype"][i]), int(c["date"][i]), float(c["v0"][i]), alt or "", msg or "",
                    tuple(sorted((md or {}).items()))))
    return out


def test_gloo_two_ranks():
    import multiprocessing as mp
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    single = CpuInboundEngine(EngineConfig.small())
    shard_fleet(single, 1, 0)
    tot, ref = [], []
    for r in range(2):
        tot.append(single.step(*fleet_batch(1000, seed=500 + r, n_dev=N_DEV), NOW, presence=False))
        ref += _block_string_keys(single.encode_block(NOW, tot[-1], boot=5))
    assert sum(o[1] for o in outs) == sum(t.n_events for t in tot)
    assert sum(o[2] for o in outs) == sum(t.n_persisted for t in tot)
    assert all(o[3] for o in outs)
    # whole events on the owner ranks: the strings crossed the exchange with the records
    got = [k for o in outs for k in o[4]]
    assert sum(1 for k in got if k[3]) > 0.8 * len(got)
    assert sorted(got) == sorted(ref)


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X GPU")
def test_numa_binding_is_safe():
    """bind_numa never leaves the process without CPUs (node -1 when the topology is unknown)."""
    from sitewhere_amd.parallel.sharding import bind_numa, gpu_numa_node
    before = os.sched_getaffinity(0)
    node = bind_numa(0)
    assert node == -1 or node == gpu_numa_node(0)
    assert os.sched_getaffinity(0)
    os.sched_setaffinity(0, before)


def test_wire_pack_is_lossless_for_every_decoded_type():
    """The 64-byte exchange form round-trips every record the decoder emits (all event types,
    control and decode-error records) -- the packing may not change any result."""
    from sitewhere_amd.models.columnar import EVENT_REC, wire_pack, wire_unpack
    from sitewhere_amd.pipeline.fleet import cpu_decode
    from pipeline_scenarios import hand_batch
    recs = [cpu_decode(*fleet_batch(3000, seed=s, n_dev=N_DEV), NOW, 2, cap=1 << 16) for s in (1, 2)]
    raw, offs = hand_batch()
    recs.append(cpu_decode(raw, offs, NOW, 2, cap=1 << 12))
    r = np.concatenate(recs)
    assert {0, 1, 2}.issubset(set(r["etype"].tolist())) and (r["etype"] >= 16).any()
    back = wire_unpack(wire_pack(r), 2)
    assert back.tobytes() == r.tobytes()
    assert EVENT_REC.itemsize == 80


def _skewed_batch(world, rank, k, n=1200):
    """Payloads of devices all owned by the other rank (every record crosses the exchange)."""
    from sitewhere_amd.models import wire
    from sitewhere_amd.pipeline.fleet import pack_messages
    heap, offs = gen_tokens("dev-", 0, N_DEV)
    lo, hi = fingerprints(heap, offs)
    theirs = np.nonzero(((hi >> np.uint64(32)) % np.uint64(world)) == (rank + 1) % world)[0]
    msgs = [wire.measurements(f"dev-{int(theirs[(k * 131 + i) % len(theirs)]):010d}", {"v": float(i)},
                              event_date=NOW - 1000 + i, alternate_id=f"sk-{rank}-{k}-{i}") for i in range(n)]
    return pack_messages(msgs)


def _gloo_skew_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # slabs of ~250 records for ~1200 records per batch: every round spills, the carry would pass
    # carry_cap (= carry_high + 2 * rec_cap) within a few rounds without the stall rule
    e = CpuInboundEngine(EngineConfig.small(world=world, rank=rank, max_msgs=1200, shuffle_slack=0.2,
                                            shuffle_pad=0))
    shard_fleet(e, world, rank)
    batches = [_skewed_batch(world, rank, k) for k in range(12)]
    empty = (np.zeros(64, np.uint8), np.zeros(1, np.uint32))
    nxt = stalls = rounds = events = 0
    peak = 0
    while True:
        if nxt < len(batches) and not e.should_stall():
            raw, offs = batches[nxt]
            nxt += 1
        else:
            stalls += nxt < len(batches)
            raw, offs = empty
        events += e.step(raw, offs, NOW, presence=False).n_events
        rounds += 1
        peak = max(peak, e.carry_count())
        left = torch.tensor([len(batches) - nxt + e.carry_count()], dtype=torch.int64)
        dist.all_reduce(left)                   # every rank runs the same number of rounds
        if int(left) == 0 or rounds > 400:
            break
    s = e.stats_dict()
    q.put((rank, events, s["shuffle_overflow"], s["shuffle_deferred"], stalls, peak, e.cfg.carry_cap, rounds))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_skewed_keys_stall_instead_of_dropping():
    """Two gloo ranks whose payloads all belong to the other rank, through slabs far smaller than a
    batch: the carry would overflow carry_cap, so the drivers feed exchange-only rounds while it is
    high (EngineBase.should_stall) -- shuffle_overflow stays 0 and every event is processed once."""
    import multiprocessing as mp
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gloo_skew_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = sorted(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(o[2] == 0 for o in outs), outs                 # nothing dropped
    assert all(o[3] > 0 for o in outs) and any(o[4] > 0 for o in outs), outs   # spilled, and stalled
    assert all(o[5] <= o[6] for o in outs), outs              # carry stayed within carry_cap
    assert sum(o[1] for o in outs) == 2 * 12 * 1200           # every event processed exactly once


def _skewed_string_batch(world, rank, k, n=800):
    """Skewed payloads (every device owned by the other rank) with 60-byte alternate ids, metadata
    on every other payload and alerts with messages."""
    from sitewhere_amd.models import wire
    from sitewhere_amd.pipeline.fleet import pack_messages
    heap, offs = gen_tokens("dev-", 0, N_DEV)
    lo, hi = fingerprints(heap, offs)
    theirs = np.nonzero(((hi >> np.uint64(32)) % np.uint64(world)) == (rank + 1) % world)[0]
    msgs = []
    for i in range(n):
        tok = f"dev-{int(theirs[(k * 131 + i) % len(theirs)]):010d}"
        alt = f"lossless-{rank}-{k:04d}-{i:05d}-".ljust(60, "x")
        md = {"site": f"s{i % 7}", "fw": f"1.{i % 5}"} if i % 2 else None
        if i % 9 == 4:
            msgs.append(wire.alert(tok, "door.open", f"door opened at gate {i} of batch {k}", event_date=NOW - 900 + i,
                                   alternate_id=alt, metadata=md))
        else:
            msgs.append(wire.measurements(tok, {"v": float(i)}, event_date=NOW - 1000 + i, alternate_id=alt,
                                          metadata=md))
    return pack_messages(msgs)


def _gloo_strings_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    from sitewhere_amd.persistence.segments import decode_block, row_strings
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # record slabs of ~260 and string slabs of ~260 x 24 bytes: the string slab fills first (each
    # record carries 60-150 bytes), so most records wait in the carry -- with their strings
    e = CpuInboundEngine(EngineConfig.small(world=world, rank=rank, max_msgs=800, shuffle_slack=0.3,
                                            shuffle_pad=0, str_bytes=24))
    shard_fleet(e, world, rank)
    batches = [_skewed_string_batch(world, rank, k) for k in range(8)]
    empty = (np.zeros(64, np.uint8), np.zeros(1, np.uint32))
    nxt = rounds = 0
    stored = []
    peak = 0
    while True:
        if nxt < len(batches) and not e.should_stall():
            raw, offs = batches[nxt]
            nxt += 1
        else:
            raw, offs = empty
        res = e.step(raw, offs, NOW, presence=False)
        if res.n_persisted:
            c = decode_block(e.encode_block(NOW, res, boot=0x77))
            for i in range(len(c["date"])):
                alt, msg, md = row_strings(c, i)
                stored.append((alt, msg, tuple(sorted(md.items()))))
        rounds += 1
        peak = max(peak, e.carry_count())
        left = torch.tensor([len(batches) - nxt + e.carry_count()], dtype=torch.int64)
        dist.all_reduce(left)
        if int(left) == 0 or rounds > 600:
            break
    s = e.stats_dict()
    q.put((rank, stored, s["shuffle_overflow"], s["shuffle_deferred"], peak, list(e.str_drops), rounds, s))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_skewed_strings_are_lossless():
    """two gloo ranks, skewed keys (every record crosses the exchange), 60-byte
    alternate ids, metadata and alert messages through string slabs far too small for a batch:
    records whose strings do not fit wait in the carry with their strings, so the owner ranks store
    every event with every string -- the same strings the decoding ranks were sent."""
    import multiprocessing as mp
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gloo_strings_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = sorted((q.get(timeout=300) for _ in range(2)), key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, stored, overflow, deferred, peak, drops, rounds, _ in outs:
        assert overflow == 0 and deferred > 0 and drops == [0, 0], (rank, overflow, deferred, drops)
    # every payload sent by either rank is stored by the other, with its strings intact
    want = {}
    for r in range(2):
        for k in range(8):
            for i in range(800):
                alt = f"lossless-{r}-{k:04d}-{i:05d}-".ljust(60, "x")
                md = tuple(sorted({"site": f"s{i % 7}", "fw": f"1.{i % 5}"}.items())) if i % 2 else ()
                msg = f"door opened at gate {i} of batch {k}" if i % 9 == 4 else ""
                want[alt] = (msg, md)
    got = {}
    for rank, stored, *_ in outs:
        for alt, msg, md in stored:
            assert alt not in got, alt                         # stored once
            got[alt] = (msg, md)
    assert got == want


def _gloo_dedup_worker(rank, world, port, q, seed_fp):
    import torch
    import torch.distributed as dist
    from sitewhere_amd.persistence.segments import decode_block, row_strings
    from sitewhere_amd.pipeline.recheck import settle_rechecks
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # a window of a few batches (it rotates twice before the replay), the store-backed filter on
    e = CpuInboundEngine(EngineConfig.small(world=world, rank=rank, max_msgs=800, dedup_slots=1 << 12,
                                            dedup_filter_ids=1 << 12, dedup_filter_gens=4))
    shard_fleet(e, world, rank)
    if seed_fp:
        # false positives on demand: the owner's filter already holds every id it will be sent (ids
        # never stored -- what a fingerprint collision is, ~1e-8 of ids in a real run)
        from sitewhere_amd.pipeline.fleet import hash64
        src = (rank - 1) % world
        e.filter_seed_begin()
        e.filter_seed(np.array([hash64(f"lossless-{src}-{k:04d}-{i:05d}-".ljust(60, "x"))
                                for k in range(6) for i in range(800)], np.uint64))
    fresh = [_skewed_string_batch(world, rank, k) for k in range(6)]
    batches = fresh + [fresh[0]]              # the first batch again, long after the window forgot it
    empty = (np.zeros(64, np.uint8), np.zeros(1, np.uint32))
    store: dict = {}                          # this rank's event store: alternate id -> times stored
    nxt = rounds = 0
    settled = {"rechecks": 0, "duplicates": 0, "injected": 0}
    while True:
        if nxt < len(batches) and not e.should_stall():
            raw, offs = batches[nxt]
            nxt += 1
        else:
            raw, offs = empty
        res = e.step(raw, offs, NOW, presence=False)
        if res.n_persisted:
            c = decode_block(e.encode_block(NOW, res, boot=0x78))
            for i in range(len(c["date"])):
                alt = row_strings(c, i)[0]
                store[alt] = store.get(alt, 0) + 1
        for k, v in settle_rechecks(e, res, lambda ids: [a in store for a in ids]).items():
            settled[k] += v
        rounds += 1
        left = torch.tensor([len(batches) - nxt + e.carry_count()], dtype=torch.int64)
        dist.all_reduce(left)
        if int(left) == 0 or rounds > 600:
            break
    s = e.stats_dict()
    q.put((rank, store, settled, s["dedup_rotations"], s["duplicates"], s["shuffle_overflow"]))
    dist.barrier()
    dist.destroy_process_group()


def _run_gloo_dedup(seed_fp):
    import multiprocessing as mp
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gloo_dedup_worker, args=(r, 2, port, q, seed_fp)) for r in range(2)]
    for p in procs:
        p.start()
    outs = sorted((q.get(timeout=300) for _ in range(2)), key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = {f"lossless-{r}-{k:04d}-{i:05d}-".ljust(60, "x") for r in range(2) for k in range(6) for i in range(800)}
    got: dict = {}
    for _, store, *_ in outs:
        for alt, n in store.items():
            assert n == 1 and alt not in got, alt                    # stored once
            got[alt] = n
    assert set(got) == want
    return outs


def test_gloo_replay_beyond_window_is_caught_on_the_owner():
    """two gloo ranks, skewed keys -- every record is decoded on one rank
    and owned by the other.  After the dedup window has rotated past the first batch, both ranks
    send it again: the owner's store-backed filter flags every replayed id (records decoded on
    another rank go through it too, their strings came along), the owner settles them by alternate
    id against its store, and all 1,600 are duplicates -- 800 caught on each rank."""
    outs = _run_gloo_dedup(False)
    for rank, store, settled, rotations, dups, overflow in outs:
        assert rotations >= 2 and overflow == 0, (rank, rotations, overflow)
        assert settled["duplicates"] == 800, (rank, settled)


def test_gloo_filter_false_positives_are_settled_and_stored_once():
    """Every fresh id a false positive (the owners' filters seeded with ids never stored): the
    owners settle each recheck by alternate id; the ids the store does not hold go back into the
    re-key carry, filter-settled, and are stored exactly once with their strings; the replay is
    still caught."""
    outs = _run_gloo_dedup(True)
    for rank, store, settled, rotations, dups, overflow in outs:
        assert settled["injected"] > 1000 and settled["duplicates"] == 800, (rank, settled)
