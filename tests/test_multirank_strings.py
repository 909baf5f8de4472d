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


def _batches():
    from sitewhere_amd.pipeline.fleet import FleetSpec, gen_payloads
    spec = FleetSpec(prefix="dev-", n_devices=N_DEV, p_location=0.25, p_alert=0.15, p_unregistered=0.0,
                     mx_per_msg=2, n_names=8, with_alternate_id=True, lat0=33.0, lon0=-85.0, span_deg=2.0,
                     p_meta=0.3)
    out = []
    for r in range(W):
        raw, offs = gen_payloads(spec, N_MSGS, NOW - 60_000, seed=900 + r)
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
        assert e.string_drops() == {"slab_full": 0, "carried": 0}
    assert len(got) == len(ref)
    with_alt = sum(1 for k in got if k[3])
    assert with_alt > 0.9 * len(got) - 100                     # nearly every device event has one
    assert sum(1 for k in got if k[5]) > 0 and sum(1 for k in got if k[4]) > 0   # metadata, messages
    assert sorted(got) == sorted(ref)


def test_string_slab_overflow_is_counted_not_corrupting():
    """A slab too small for the step's strings drops whole records' strings (counted); the rows
    are still stored, and every string that is stored is intact."""
    import torch
    from sitewhere_amd.pipeline.config import EngineConfig
    from sitewhere_amd.pipeline.gpu_engine import GpuInboundEngine
    batches = _batches()
    g = [GpuInboundEngine(EngineConfig.small(world=W, rank=r, str_bytes=2), device="cuda:0") for r in range(W)]
    for r, e in enumerate(g):
        _register(e, W, r)
    bufs = []                                   # the device batches stay alive until processed
    for e, (raw, offs) in zip(g, batches):
        bufs.append((torch.from_numpy(raw).cuda(), torch.from_numpy(offs.view(np.int32)).cuda()))
        e.prepare(*bufs[-1], len(offs) - 1, NOW, out_to_device=True)
        e.phase_decode()
    torch.cuda.synchronize()
    for q in range(W):
        for r in range(W):
            g[q].recv_slab(r).copy_(g[r].send_slab(q))
            g[q].t["recv_cnt"][r] = g[r].send_count(q)
        g[q].loopback_strings(g)
    alts = set()
    for (raw, _), e in zip(batches, g):
        e.phase_process()
        torch.cuda.synchronize()
        res = e.collect(e._last_sel, raw, from_device=True)
        keys = _row_keys(e.encode_block(NOW, res, boot=0x5))
        assert e.string_drops()["slab_full"] > 0
        alts |= {k[3] for k in keys if k[3]}
    # stored alternate ids are well-formed "<16 hex>-<8 hex>[:k]"
    for a in alts:
        base = a.split(":")[0]
        assert len(base) == 25 and base[16] == "-", a
