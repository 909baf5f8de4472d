"""Lossless records on several ranks: a record's strings (alternate id, metadata, alert message) sit
in the raw batch of the rank that decoded it, and the re-key exchange carries them to the owner
rank in per-destination byte slabs (``SwEngineArgs.send_str``; ``k_part_write`` / ``k_unpack``).
W GPU engine shards in one process, exchanging by plain copies (loopback), must store the same
events with the same strings as one single-rank engine that processes every batch itself."""
from __future__ import annotations

import numpy as np
import pytest

from tests.conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs an MI355X GPU")]

W = 2
N_DEV = 4096
N_MSGS = 3000
NOW = 1_700_000_300_000


def _register(e, world, rank):
    from sitewhere_amd.pipeline.fleet import fingerprints, gen_tokens
    heap, offs = gen_tokens("dev-", 0, N_DEV)
    lo, hi = fingerprints(heap, offs)
    dev = e.register_devices(lo, hi)              # replicated registry (tests/test_multirank.py)
    e.set_assignments(dev, dev, customer=dev % 7, area=dev % 5, asset=dev % 3)


def _batches(seed=900):
    from sitewhere_amd.pipeline.fleet import FleetSpec, gen_payloads
    spec = FleetSpec(prefix="dev-", n_devices=N_DEV, p_location=0.25, p_alert=0.15, p_unregistered=0.0,
                     mx_per_msg=2, n_names=8, with_alternate_id=True, lat0=33.0, lon0=-85.0, span_deg=2.0,
                     p_meta=0.3)
    out = []
    for r in range(W):
        raw, offs = gen_payloads(spec, N_MSGS, NOW - 60_000, seed=seed + r)
        out.append((np.concatenate([raw, np.zeros(64, np.uint8)]), offs))
    return out


def _row_keys(block) -> list:
    """(type, date, value, alternate id, message, metadata) of every row of a block."""
    from sitewhere_amd.persistence.segments import decode_block, row_strings
    c = decode_block(block)
    keys = []
    for i in range(len(c["etype"])):
        alt, msg, md = row_strings(c, i)
        keys.append((int(c["etype"][i]), int(c["date"][i]), float(c["v0"][i]), alt or "", msg or "",
                     tuple(sorted((md or {}).items()))))
    return keys


def test_strings_cross_the_exchange():
    import torch
    from sitewhere_amd.pipeline.config import EngineConfig
    from sitewhere_amd.pipeline.gpu_engine import GpuInboundEngine
    batches = _batches()
    # reference: one rank processes every batch
    one = GpuInboundEngine(EngineConfig.small(), device="cuda:0")
    _register(one, 1, 0)
    ref = []
    for raw, offs in batches:
        res = one.step(raw, offs, NOW, presence=False)
        ref += _row_keys(one.encode_block(NOW, res, boot=0x5))
    # W shards, loopback exchange
    g = [GpuInboundEngine(EngineConfig.small(world=W, rank=r), device="cuda:0") for r in range(W)]
    for r, e in enumerate(g):
        _register(e, W, r)
    bufs = []
    for e, (raw, offs) in zip(g, batches):
        rd = torch.from_numpy(raw).cuda()
        od = torch.from_numpy(offs.view(np.int32)).cuda()
        bufs.append((rd, od))
        e.prepare(rd, od, len(offs) - 1, NOW, out_to_device=True)
        e.phase_decode()
    torch.cuda.synchronize()
    for q in range(W):
        for r in range(W):
            g[q].recv_slab(r).copy_(g[r].send_slab(q))
            g[q].t["recv_cnt"][r] = g[r].send_count(q)
        g[q].loopback_strings(g)
    got = []
    for (raw, _), e in zip(batches, g):
        e.phase_process()
        torch.cuda.synchronize()
        res = e.collect(e._last_sel, raw, from_device=True)
        got += _row_keys(e.encode_block(NOW, res, boot=0x5))
        assert e.string_drops() == {"oversize": 0}
    assert len(got) == len(ref)
    with_alt = sum(1 for k in got if k[3])
    assert with_alt > 0.9 * len(got) - 100                     # nearly every device event has one
    assert sum(1 for k in got if k[5]) > 0 and sum(1 for k in got if k[4]) > 0   # metadata, messages
    assert sorted(got) == sorted(ref)


def test_small_string_slabs_defer_records_with_their_strings():
    """String slabs far too small for a step's strings (2 bytes per record slot) take a prefix of
    each destination's records; the rest wait in the carry with their strings (the carry heap) and
    go in later rounds -- nothing is dropped.  Every round's slabs (records, string bytes, refs) and
    carry (records, refs, heap) are byte-identical to the oracle's (``CpuInboundEngine.partition``),
    and after the drain rounds the shards have stored exactly the single-rank engine's rows, every
    string included."""
    import torch
    from sitewhere_amd.models.columnar import EVENT_REC, STR_REF, wire_pack
    from sitewhere_amd.pipeline.config import EngineConfig
    from sitewhere_amd.pipeline.cpu_engine import CpuInboundEngine
    from sitewhere_amd.pipeline.gpu_engine import GpuInboundEngine
    batches = _batches()
    one = GpuInboundEngine(EngineConfig.small(), device="cuda:0")
    _register(one, 1, 0)
    ref = []
    for raw, offs in batches:
        res = one.step(raw, offs, NOW, presence=False)
        ref += _row_keys(one.encode_block(NOW, res, boot=0x5))
    cfg = dict(str_bytes=2)
    g = [GpuInboundEngine(EngineConfig.small(world=W, rank=r, **cfg), device="cuda:0") for r in range(W)]
    c = [CpuInboundEngine(EngineConfig.small(world=W, rank=r, **cfg)) for r in range(W)]
    for r in range(W):
        _register(g[r], W, r)
        _register(c[r], W, r)
    cap, S = g[0].cfg.str_cap, g[0].cfg.shuf_cap
    empty = (np.zeros(64, np.uint8), np.zeros(1, np.uint32))
    got, deferred = [], 0
    for k in range(80):
        bs = batches if k == 0 else [empty] * W
        keep = []
        for e, (raw, offs) in zip(g, bs):
            keep.append((torch.from_numpy(raw).cuda(), torch.from_numpy(offs.view(np.int32)).cuda()))
            e.prepare(*keep[-1], len(offs) - 1, NOW, out_to_device=True)
            e.phase_decode()
        torch.cuda.synchronize()
        for r, (e, (raw, offs)) in enumerate(zip(c, bs)):
            recs, _ = e.decode_phase(raw, offs, NOW)
            rw = np.asarray(raw, np.uint8)
            send, cnt, index, nc = e.partition(recs, with_index=True, spans=e._dec_spans, raw=rw)
            sp, buf, used = e._pack_strings(send, index, nc, e._dec_spans, rw)
            ge = g[r]
            p = ge._last_send_par
            assert ge.send_cnts[p].cpu().numpy().tolist() == cnt.tolist(), (k, r)
            assert ge.send_str_cnts[p].cpu().numpy().tolist() == used.tolist(), (k, r)
            gsp = ge.send_spans[p].cpu().numpy().view(STR_REF).reshape(W, S)
            gst = ge.send_strs[p].cpu().numpy().reshape(W, cap)
            for q in range(W):
                n = int(cnt[q])
                assert np.array_equal(ge.send_slab(q).cpu().numpy()[:n * 64], wire_pack(send[q, :n]).view(np.uint8))
                assert np.array_equal(gsp[q, :n], sp[q, :n]), (k, r, q)
                assert np.array_equal(gst[q, :int(used[q])], buf[q * cap:q * cap + int(used[q])]), (k, r, q)
            cp = ge._carry_par
            n = int(ge.t["n_carry"][cp].item())
            assert n == len(e.carry)
            assert np.array_equal(ge.carry_bufs[cp][:n * EVENT_REC.itemsize].cpu().numpy(), e.carry.view(np.uint8))
            assert np.array_equal(ge.carry_spans[cp][:n * STR_REF.itemsize].cpu().numpy().view(STR_REF), e.carry_sp)
            nb = int(ge.t["n_carry_str"][cp].item())
            assert nb == len(e.carry_heap)
            assert np.array_equal(ge.carry_strs[cp][:nb].cpu().numpy(), e.carry_heap)
            deferred += n
        for q in range(W):
            for r in range(W):
                g[q].recv_slab(r).copy_(g[r].send_slab(q))
                g[q].t["recv_cnt"][r] = g[r].send_count(q)
            g[q].loopback_strings(g)
        for (raw, _), e in zip(bs, g):
            e.phase_process()
            torch.cuda.synchronize()
            res = e.collect(e._last_sel, raw, from_device=True)
            got += _row_keys(e.encode_block(NOW, res, boot=0x5))
        if k and not any(len(e.carry) for e in c):
            break
    assert deferred > 0 and not any(len(e.carry) for e in c)
    for e in g:
        assert e.string_drops() == {"oversize": 0}
        assert e.stats_dict()["shuffle_overflow"] == 0
    assert len(got) == len(ref)
    assert sorted(got) == sorted(ref)


def _gpu_round(g, bs, packages=None):
    """One loopback round of the W shards: decode + partition, slab copies, process; results.
    ``packages``: a list that gets each shard's recheck packages from its reject snapshot
    (``k_reject_refs``, what ``bench.py``'s pipelined path settles)."""
    import torch
    keep = []
    for e, (raw, offs) in zip(g, bs):
        keep.append((torch.from_numpy(raw).cuda(), torch.from_numpy(offs.view(np.int32)).cuda()))
        e.prepare(*keep[-1], len(offs) - 1, NOW, out_to_device=True)
        e.phase_decode()
    torch.cuda.synchronize()
    for q in range(W):
        for r in range(W):
            g[q].recv_slab(r).copy_(g[r].send_slab(q))
            g[q].t["recv_cnt"][r] = g[r].send_count(q)
        g[q].loopback_strings(g)
    out = []
    for (raw, offs), e, dev in zip(bs, g, keep):
        e.phase_process()
        torch.cuda.synchronize()
        if packages is not None:
            from sitewhere_amd.pipeline.recheck import unpack_rechecks
            cnt, _ = e.reject_refs_async(e._last_sel, dev[0], dev[1], len(offs) - 1)
            torch.cuda.synchronize()
            n_ref, n_b = (int(v) for v in cnt[:2].cpu())
            refs, comp = e.reject_snapshot(e._last_sel, n_ref, n_b)
            packages.append(unpack_rechecks(refs.copy(), comp.copy()))
        out.append(e.collect(e._last_sel, raw, from_device=True))
    return out


def test_gpu_rechecks_are_settled_by_alternate_id_on_the_owner():
    """Several ranks, store-backed dedup: the owner's filter sees records decoded on
    another rank too (their strings came along), and the owner settles each recheck by its
    alternate id (``pipeline/recheck.py``).  Filters seeded with every fresh id (ids never stored:
    false positives on demand) make each fresh id a recheck: those are re-injected into the re-key
    carry, filter-settled, and stored exactly once with their strings.  A replay after the window is
    reset is caught: every replayed id comes back as a recheck the store holds, a duplicate."""
    from sitewhere_amd.pipeline.config import EngineConfig
    from sitewhere_amd.pipeline.fleet import cpu_decode
    from sitewhere_amd.pipeline.gpu_engine import GpuInboundEngine
    from sitewhere_amd.pipeline.recheck import settle_rechecks
    g = [GpuInboundEngine(EngineConfig.small(world=W, rank=r, dedup_filter_ids=1 << 15), device="cuda:0")
         for r in range(W)]
    fresh = np.concatenate([cpu_decode(raw, offs, NOW)["alt_hash"] for seed in (900, 950)
                            for raw, offs in _batches(seed)])
    for r, e in enumerate(g):
        _register(e, W, r)
        e.filter_seed_begin()
        e.filter_seed(fresh[fresh != 0])
    stores = [dict() for _ in range(W)]
    totals = {"rechecks": 0, "duplicates": 0, "injected": 0}
    empty = (np.zeros(64, np.uint8), np.zeros(1, np.uint32))

    packaged = {"same": 0}

    def same_rechecks(pkg, rc):
        # the snapshot's packages hold the rechecks collect() gathers, strings included
        from sitewhere_amd.pipeline.recheck import alternate_ids
        pr, ps, ph, lost = pkg
        assert lost == 0
        if rc is None:
            assert len(pr) == 0
            return

        def rows(r, s, h):
            msg = [bytes(h[int(x["aux2_off"]):int(x["aux2_off"]) + int(x["aux2_len"])]) if x["etype"] == 2 else b""
                   for x in r]
            meta = [bytes(h[int(y["meta_off"]):int(y["meta_off"]) + int(y["meta_len"])]) for y in s]
            return sorted(zip(r["alt_hash"].tolist(), r["event_date"].tolist(), r["etype"].tolist(),
                              alternate_ids(s, h), meta, msg))
        assert rows(pr, ps, ph) == rows(*rc)
        packaged["same"] += len(pr)

    def run(bs):
        for k in range(20):
            pk = []
            res = _gpu_round(g, bs if k == 0 else [empty] * W, packages=pk)
            for r, (e, x) in enumerate(zip(g, res)):
                same_rechecks(pk[r], x.recheck)
                for key in _row_keys(e.encode_block(NOW, x, boot=0x5)):
                    if key[3]:
                        stores[r][key[3]] = stores[r].get(key[3], 0) + 1
                for kk, v in settle_rechecks(e, x, lambda ids, s=stores[r]: [a in s for a in ids]).items():
                    totals[kk] += v
            if not any(e.carry_count() for e in g):
                return
        raise AssertionError("carry did not drain")

    first, second = _batches(900), _batches(950)
    run(first)
    run(second)
    assert totals["injected"] > 1000 and totals["duplicates"] == 0, totals
    assert packaged["same"] == totals["rechecks"], packaged
    stored = {}
    for s in stores:
        for a, n in s.items():
            assert n == 1 and a not in stored, a
            stored[a] = n
    n_ids = len(stored)
    for e in g:
        e.reset_dedup()
    before = dict(totals)
    run(first)
    assert totals["duplicates"] - before["duplicates"] == totals["rechecks"] - before["rechecks"] > 1000, totals
    assert sum(len(s) for s in stores) == n_ids and all(n == 1 for s in stores for n in s.values())
    for e in g:
        assert e.string_drops() == {"oversize": 0}


def test_gpu_checkpoint_keeps_the_carry_strings():
    """An engine checkpoint taken while records (and their strings) wait in the re-key carry
    restores them into fresh shards: the drained rows equal an uninterrupted run's."""
    from sitewhere_amd.pipeline.config import EngineConfig
    from sitewhere_amd.pipeline.gpu_engine import GpuInboundEngine
    batches = _batches(977)
    empty = (np.zeros(64, np.uint8), np.zeros(1, np.uint32))

    def shards():
        g = [GpuInboundEngine(EngineConfig.small(world=W, rank=r, str_bytes=2), device="cuda:0") for r in range(W)]
        for r, e in enumerate(g):
            _register(e, W, r)
        return g

    def drain(g, rows):
        for k in range(80):
            for (raw, _), e, x in zip([empty] * W, g, _gpu_round(g, [empty] * W)):
                rows += _row_keys(e.encode_block(NOW, x, boot=0x5))
            if not any(e.carry_count() for e in g):
                return rows
        raise AssertionError("carry did not drain")

    # uninterrupted
    a = shards()
    ref = []
    for e, x in zip(a, _gpu_round(a, batches)):
        ref += _row_keys(e.encode_block(NOW, x, boot=0x5))
    drain(a, ref)
    # checkpoint right after the first round (most records still in the carry), restore, drain
    b = shards()
    got = []
    for e, x in zip(b, _gpu_round(b, batches)):
        got += _row_keys(e.encode_block(NOW, x, boot=0x5))
    assert sum(e.carry_count() for e in b) > 0
    states = [e.checkpoint_state() for e in b]
    c = shards()
    for e, st in zip(c, states):
        e.restore_state(st, include_store=False)
    assert [e.carry_count() for e in c] == [e.carry_count() for e in b]
    drain(c, got)
    assert sorted(got) == sorted(ref)
