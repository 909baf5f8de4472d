"""MI355X block index trailers (csrc/hip/swindex.hip) and the radix sort behind the persist clustering,
against their host references: numpy's stable argsort, and the C++ trailer builder
(csrc/native/swindex.cpp swseg_index_append) run on the GPU's own block -- byte for byte."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

from tests.conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]


@pytest.mark.parametrize("n,bits", [(0, 8), (1, 8), (4095, 21), (4096, 16), (70_001, 21), (1_100_000, 21),
                                    (300_000, 11), (200_000, 32)])
def test_radix_sort_stable(n, bits):
    import torch
    from sitewhere_amd._native import gpu
    lib = gpu()
    d = torch.device("cuda", 0)
    rng = np.random.default_rng(n + bits)
    cap = max(n, 1) + 777
    keys = rng.integers(0, 1 << min(bits, 31), n, dtype=np.int64).astype(np.uint32)
    if bits == 32:
        keys |= (rng.integers(0, 2, n) << 31).astype(np.uint32)
    keys[: n // 3] = keys[0] if n else 0                      # a heavy duplicate run: stability matters
    vals = np.arange(n, dtype=np.uint32)
    kb = torch.zeros(2 * cap, dtype=torch.int32, device=d)
    vb = torch.zeros(2 * cap, dtype=torch.int32, device=d)
    if n:
        kb[:n] = torch.from_numpy(keys.view(np.int32)).to(d)
        vb[:n] = torch.from_numpy(vals.view(np.int32)).to(d)
    hist = torch.zeros(int(lib.sw_radix_tmp_words(cap)), dtype=torch.int32, device=d)
    nt = torch.tensor([n], dtype=torch.int32, device=d)
    s = torch.cuda.current_stream(d)
    P = ctypes.c_void_p
    buf = lib.sw_radix_sort_u32(P(kb.data_ptr()), P(vb.data_ptr()), P(nt.data_ptr()), cap, bits, P(hist.data_ptr()),
                                None, P(s.cuda_stream))
    assert buf in (0, 1)
    s.synchronize()
    gk = kb[buf * cap:buf * cap + n].cpu().numpy().view(np.uint32)
    gv = vb[buf * cap:buf * cap + n].cpu().numpy().view(np.uint32)
    masked = keys & np.uint32((1 << bits) - 1 if bits < 32 else 0xFFFFFFFF)
    order = np.argsort(masked, kind="stable")
    assert np.array_equal(gv, vals[order])
    assert np.array_equal(gk, keys[order])


def _engines(n_dev=3000, asset_mod=3, **kw):
    from sitewhere_amd.pipeline.config import EngineConfig
    from sitewhere_amd.pipeline.cpu_engine import CpuInboundEngine
    from sitewhere_amd.pipeline.engine_base import Zone, ZoneTest
    from sitewhere_amd.pipeline.fleet import fingerprints, gen_tokens
    from sitewhere_amd.pipeline.gpu_engine import GpuInboundEngine
    cfg = dict(max_msgs=8192, gen_cap=8192, max_devices=4096, max_assignments=4096, store_cap=1 << 14,
               dedup_slots=1 << 15, name_slots=1 << 10, names_cap=1024)
    cfg.update(kw)
    g = GpuInboundEngine(EngineConfig.small(**cfg), device="cuda:0")
    c = CpuInboundEngine(EngineConfig.small(**cfg))
    heap, offs = gen_tokens("dev-", 0, n_dev)
    lo, hi = fingerprints(heap, offs)
    zones = [Zone("z", [(33.0, -85.0), (33.0, -84.0), (34.0, -84.0), (34.0, -85.0)])]
    for e in (g, c):
        d = e.register_devices(lo, hi)
        asg = np.random.default_rng(9).permutation(len(d)).astype(np.int32)
        e.set_assignments(asg, d, customer=asg % 7, area=asg % 5, asset=asg % asset_mod)
        e.set_zone_rules(zones, [ZoneTest("z", "inside", "zone.enter", 2)])
    return g, c


def _strip_trailer(blk: np.ndarray) -> np.ndarray:
    """The block without its trailer (flag cleared, bytes = end of the pages, header re-sealed)."""
    from sitewhere_amd.persistence import segments as sg
    h = blk[:64].view(sg.HDR)[0]
    toff = sg.trailer_offset(blk)
    out = blk[:toff].copy()
    hv = out[:64].view(sg.HDR)
    hv["flags"] = 0
    hv["bytes"] = toff
    sg.seal(out, int(h["first_seq"]), int(h["recv_ms"]), int(h["boot"]), int(h["rank"]), int(h["world"]))
    return out


@pytest.mark.parametrize("asset_mod", [3, 9000])
def test_gpu_trailer_matches_cpu_builder(asset_mod):
    """Four engine steps (the ring wraps): the GPU block's trailer == the C++ builder's trailer over the
    same block, byte for byte; the blocks' rows equal the oracle's (same clustered order)."""
    from sitewhere_amd.persistence import segments as sg
    from sitewhere_amd.pipeline.fleet import FleetSpec, gen_payloads
    from tests.test_block_index import check_trailer
    g, c = _engines(asset_mod=asset_mod)
    spec = FleetSpec(prefix="dev-", n_devices=3000, p_location=0.3, p_alert=0.05, p_unregistered=0.01,
                     mx_per_msg=2, with_alternate_id=True, lat0=32.8, lon0=-85.2, span_deg=1.5, p_meta=0.2)
    now = 1_700_000_001_000
    for b in range(4):
        raw, off = gen_payloads(spec, 3500, now - 30_000, seed=b + 1)
        raw = np.concatenate([raw, np.zeros(64, np.uint8)])
        rg = g.step(raw, off, now + b, presence=False)
        rc = c.step(raw, off, now + b, presence=False)
        np.testing.assert_array_equal(rg.out["assignment"], rc.out["assignment"])
        bg = g.encode_block(now + b, rg, boot=0xabc)
        assert sg.verify(bg) == 0
        ref = sg.index_block(_strip_trailer(bg), g.ctx_table())
        assert len(ref) == len(bg), (len(ref), len(bg))
        if not np.array_equal(ref, bg):
            bad = np.nonzero(ref != bg)[0]
            pytest.fail(f"step {b}: {len(bad)} trailer bytes differ, first at {bad[0] - sg.trailer_offset(bg)}")
        check_trailer(bg, g.ctx_table())


@pytest.mark.parametrize("n_cust", [97, 1])
def test_gpu_trailer_large_step(n_cust):
    """A 1M-payload step at the bench shape (1M assignments, 97 customers, 31 areas, 1009 assets):
    the trailer equals the C++ builder's.  With one customer its keys hold ~750K rows (733 chunks:
    the partials fold in two rounds)."""
    from sitewhere_amd.persistence import segments as sg
    from sitewhere_amd.pipeline.config import EngineConfig
    from sitewhere_amd.pipeline.fleet import FleetSpec, fingerprints, gen_payloads, gen_tokens
    from sitewhere_amd.pipeline.gpu_engine import GpuInboundEngine
    n_dev = 1 << 20
    cfg = EngineConfig(max_msgs=1 << 20, rec_cap=(1 << 20) + 4096, gen_cap=1 << 19, max_devices=n_dev + 4096,
                       max_assignments=n_dev + 4096, store_cap=1 << 22, dedup_slots=1 << 22, name_slots=1 << 12,
                       state_slots=1 << 24)
    g = GpuInboundEngine(cfg, device="cuda:0")
    heap, offs = gen_tokens("dev-", 0, n_dev)
    lo, hi = fingerprints(heap, offs)
    d = g.register_devices(lo, hi)
    g.set_assignments(d, d, customer=d % n_cust, area=d % 31, asset=d % 1009)
    spec = FleetSpec(prefix="dev-", n_devices=n_dev, p_location=0.25, p_alert=0.05, p_unregistered=0.005,
                     with_alternate_id=True, lat0=33.0, lon0=-85.0, span_deg=2.0, p_meta=0.1)
    now = 1_700_000_001_000
    for k in range(3):          # consecutive large steps: the build's scratch re-arms between them
        raw, off = gen_payloads(spec, 1 << 20, now - 30_000, seed=7 + k)
        raw = np.concatenate([raw, np.zeros(64, np.uint8)])
        rg = g.step(raw, off, now + k, presence=False)
        bg = g.encode_block(now + k, rg, boot=0xabc)
        assert sg.verify(bg) == 0
        ref = sg.index_block(_strip_trailer(bg), g.ctx_table())
        if not np.array_equal(ref, bg):
            bad = np.nonzero(ref != bg)[0] if len(ref) == len(bg) else [len(ref), len(bg)]
            pytest.fail(f"step {k}: trailer differs from the C++ builder ({len(bad)} bytes, first {bad[0]})")
    toff = sg.trailer_offset(bg)
    tr = sg.parse_trailer(bg[toff:])
    assert tr["n_alt"] > 1_000_000 - 20_000
    assert [int(x) for x in tr["n_keys"]][:2] == [n_cust * 3, 31 * 3]    # measurement / location / alert
    # index bytes per row (the disk cost of the indexes)
    assert (len(bg) - toff) / rg.n_persisted < 5.0


def test_gpu_framed_blocks_trailers_match_cpu_builder():
    """The service tenant's path at the 1M shape: overlapped ``submit_framed`` steps from pinned
    zero-copy records with blocks encoded on the GPU (``encode_blocks``), fresh alternate ids per
    record -- every returned block's trailer equals the C++ builder's over the same block, and every
    stored id is found through it."""
    from sitewhere_amd.persistence import segments as sg
    from sitewhere_amd.pipeline.bus_io import RawBatchRecord, parse_raw_batch
    from sitewhere_amd.pipeline.config import EngineConfig
    from sitewhere_amd.pipeline.fleet import FleetSpec, fingerprints, gen_payloads, gen_tokens, stamp_alt_epoch
    from sitewhere_amd.pipeline.framing import varint_lengths
    from sitewhere_amd.pipeline.gpu_engine import GpuInboundEngine
    n_dev = 1 << 20
    cfg = EngineConfig(max_msgs=1 << 20, rec_cap=(1 << 20) + 4096, gen_cap=1 << 19, max_devices=n_dev + 65536,
                       max_assignments=n_dev + 65536, store_cap=1 << 23, dedup_slots=1 << 22, name_slots=1 << 12,
                       state_slots=1 << 24, dedup_filter_ids=1 << 24, dedup_filter_gens=4)
    g = GpuInboundEngine(cfg, device="cuda:0")
    heap, offs = gen_tokens("dev-", 0, n_dev)
    lo, hi = fingerprints(heap, offs)
    d = g.register_devices(lo, hi)
    g.set_assignments(d, d)
    g.encode_blocks, g.block_boot = True, 0x5eed
    spec = FleetSpec(prefix="dev-", n_devices=n_dev, p_location=0.25, p_alert=0.05, p_unregistered=0.005,
                     with_alternate_id=True)
    now = 1_700_000_001_000
    base = [gen_payloads(spec, 1 << 20, now - 30_000, seed=11 + b) for b in range(3)]
    recs, got = [], []
    for k in range(6):
        raw, off = base[k % 3]
        raw = np.concatenate([raw, np.zeros(64, np.uint8)])
        stamp_alt_epoch(raw, off, (0x50AC << 48) | k)
        rec = RawBatchRecord(raw[:int(off[-1])], varint_lengths(off), len(off) - 1, pinned=True)
        recs.append(rec)
        got += g.submit_framed(parse_raw_batch(rec.buf.numpy()[:rec.value_len]), now + k, token=k, presence=False)
    got += g.drain_framed()
    assert [t for t, _ in got] == list(range(6))
    for k, res in got:
        blk = np.ascontiguousarray(res.block)
        assert sg.verify(blk) == 0
        ref = sg.index_block(_strip_trailer(blk), g.ctx_table())
        if not np.array_equal(ref, blk):
            n = min(len(ref), len(blk))
            bad = np.nonzero(ref[:n] != blk[:n])[0]
            pytest.fail(f"step {k}: GPU trailer differs from the C++ builder (lengths {len(ref)} / {len(blk)}, "
                        f"{len(bad)} bytes, first at trailer byte {bad[0] - sg.trailer_offset(blk) if len(bad) else None})")
