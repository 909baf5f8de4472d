"""MI355X durable-block encoder (csrc/hip/swseg.hip k_seg_encode) against the CPU encoder
(csrc/native/swseg.cpp swseg_encode): the blocks must be identical byte for byte, at page-boundary
sizes, across the event ring's wrap, with decimal exceptions, and for 2M rows (look-back over ~2000
workgroups).  Then a whole engine step: the GPU block of a step equals the CPU oracle engine's block
of the same batch."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

from tests.conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]


def _encode_gpu(rows, v2, alt, cap=None, c0=0):
    import torch
    from sitewhere_amd._native import gpu
    from sitewhere_amd.models.columnar import OUT_REC
    from sitewhere_amd.persistence.segments import PAGE_ROWS, max_block_bytes
    lib = gpu()
    n = len(rows)
    cap = cap or max(n, 1)
    d = torch.device("cuda", 0)
    ring_v2 = torch.zeros(cap, dtype=torch.float64, device=d)
    ring_alt = torch.zeros(cap, dtype=torch.int64, device=d)
    idx = torch.from_numpy((c0 + np.arange(n)) % cap).to(d)
    ring_v2[idx] = torch.from_numpy(np.ascontiguousarray(v2, np.float64)).to(d)
    ring_alt[idx] = torch.from_numpy(np.ascontiguousarray(alt, np.uint64).view(np.int64)).to(d)
    max_rows = max(n, 1) + 3000
    out_rows = torch.zeros(max_rows * OUT_REC.itemsize, dtype=torch.uint8, device=d)
    if n:
        out_rows[:n * OUT_REC.itemsize] = torch.from_numpy(np.ascontiguousarray(rows, OUT_REC).view(np.uint8)).to(d)
    cursor = torch.tensor([c0 + n, c0], dtype=torch.int64, device=d)
    bcap = max_block_bytes(max_rows)
    pages = -(-max_rows // PAGE_ROWS)
    blk = torch.zeros(bcap, dtype=torch.uint8, device=d)
    state = torch.zeros(pages + 4, dtype=torch.int64, device=d)
    s = torch.cuda.current_stream(d)
    rc = lib.sw_seg_encode(ctypes.c_void_p(out_rows.data_ptr()), ctypes.c_void_p(ring_v2.data_ptr()),
                           ctypes.c_void_p(ring_alt.data_ptr()), cap, ctypes.c_void_p(cursor.data_ptr()),
                           ctypes.c_void_p(blk.data_ptr()), bcap, ctypes.c_void_p(state.data_ptr()), pages,
                           ctypes.c_void_p(s.cuda_stream))
    assert rc == 0
    s.synchronize()
    nb, err, first = (int(x) for x in state[pages + 1:pages + 4].cpu().numpy())
    assert err == 0 and 0 < nb <= bcap, (nb, err)
    assert first == c0
    return blk[:nb].cpu().numpy()


@pytest.mark.parametrize("n,c0,full", [(0, 0, False), (1, 0, False), (1023, 0, False), (1024, 0, False),
                                       (1025, 5, False), (70_000, 0, True), (70_000, 60_000, False),
                                       (2_000_000, 0, False)])
def test_gpu_block_matches_cpu(n, c0, full):
    from sitewhere_amd.persistence import segments as sg
    from tests.test_segments import synth_rows
    rows, v2, alt = synth_rows(n, seed=n + c0, full_precision=full)
    cap = None if c0 == 0 else 100_000
    g = _encode_gpu(rows, v2, alt, cap=cap, c0=c0)
    c = sg.encode_block(rows, v2, alt)
    assert len(g) == len(c)
    if not np.array_equal(g, c):
        bad = np.nonzero(g != c)[0]
        pytest.fail(f"{len(bad)} bytes differ, first at {bad[0]} of {len(c)}")
    sg.seal(g, c0, 1, 2, 0, 1)
    assert sg.verify(g) == 0


def test_gpu_engine_step_block_matches_oracle():
    import numpy as np
    from sitewhere_amd.persistence import segments as sg
    from sitewhere_amd.pipeline.config import EngineConfig
    from sitewhere_amd.pipeline.cpu_engine import CpuInboundEngine
    from sitewhere_amd.pipeline.engine_base import Zone, ZoneTest
    from sitewhere_amd.pipeline.fleet import FleetSpec, fingerprints, gen_payloads, gen_tokens
    from sitewhere_amd.pipeline.gpu_engine import GpuInboundEngine
    cfg = dict(max_msgs=8192, gen_cap=8192, max_devices=4096, max_assignments=4096, store_cap=1 << 14,
               dedup_slots=1 << 15, name_slots=1 << 10, names_cap=1024)
    g = GpuInboundEngine(EngineConfig.small(**cfg), device="cuda:0")
    c = CpuInboundEngine(EngineConfig.small(**cfg))
    heap, offs = gen_tokens("dev-", 0, 3000)
    lo, hi = fingerprints(heap, offs)
    zones = [Zone("z", [(33.0, -85.0), (33.0, -84.0), (34.0, -84.0), (34.0, -85.0)])]
    for e in (g, c):
        d = e.register_devices(lo, hi)
        e.set_assignments(d, d, customer=d % 7, area=d % 5, asset=d % 3)
        e.set_zone_rules(zones, [ZoneTest("z", "inside", "zone.enter", 2)])
    spec = FleetSpec(prefix="dev-", n_devices=3000, p_location=0.3, p_alert=0.05, p_unregistered=0.01,
                     mx_per_msg=2, with_alternate_id=True, lat0=32.8, lon0=-85.2, span_deg=1.5)
    now = 1_700_000_001_000
    for b in range(4):          # several steps: the ring wraps (store_cap 16K, ~7K rows per step)
        raw, off = gen_payloads(spec, 3500, now - 30_000, seed=b + 1)
        raw = np.concatenate([raw, np.zeros(64, np.uint8)])
        rg = g.step(raw, off, now + b, presence=False)
        rc = c.step(raw, off, now + b, presence=False)
        assert rg.n_persisted == rc.n_persisted > 0
        bg = g.encode_block(now + b, rg, boot=0xabc)
        bc = c.encode_block(now + b, rc, boot=0xabc)
        cg, cc = sg.decode_block(bg), sg.decode_block(bc)
        assert cg["header"] == cc["header"]
        for k in cg:
            if k not in ("header", "name"):
                np.testing.assert_array_equal(cg[k], cc[k], err_msg=f"step {b}: column {k}")
        # name ids are engine-local dense ids (the GPU assigns them in arrival order): same names
        gi = {i: h for h, i in g.intern_table().items()}
        ci = {i: h for h, i in c.intern_table().items()}
        to_hash = lambda ids, inv: [inv.get(int(i), -1) if i != 0xFFFF else -1 for i in ids]  # noqa: E731
        assert to_hash(cg["name"], gi) == to_hash(cc["name"], ci), f"step {b}: names differ"
        cols = cg
        np.testing.assert_array_equal(cols["date"], rc.out["event_date"])
        np.testing.assert_array_equal(cols["v0"].view(np.uint64), rc.out["v0"].view(np.uint64))
        assert cols["header"]["first_seq"] == rc.first_seq


def test_gpu_reject_snapshot_routes_like_host():
    """k_reject_refs + compact payload copies -> native routing equals routing the CPU oracle's
    rejects against the raw batch (unregistered devices, registrations, acks; duplicates dropped)."""
    import torch
    from sitewhere_amd.pipeline import routing
    from sitewhere_amd.pipeline.config import EngineConfig
    from sitewhere_amd.pipeline.cpu_engine import CpuInboundEngine
    from sitewhere_amd.pipeline.fleet import FleetSpec, fingerprints, gen_payloads, gen_tokens
    from sitewhere_amd.pipeline.gpu_engine import GpuInboundEngine
    cfg = dict(max_msgs=8192, gen_cap=8192, max_devices=4096, max_assignments=4096, store_cap=1 << 15,
               dedup_slots=1 << 15, name_slots=1 << 10, names_cap=1024)
    g = GpuInboundEngine(EngineConfig.small(**cfg), device="cuda:0")
    c = CpuInboundEngine(EngineConfig.small(**cfg))
    heap, offs = gen_tokens("dev-", 0, 3000)
    lo, hi = fingerprints(heap, offs)
    for e in (g, c):
        d = e.register_devices(lo, hi)
        e.set_assignments(d, d)
    spec = FleetSpec(prefix="dev-", n_devices=3000, p_unregistered=0.03, mx_per_msg=2, with_alternate_id=True,
                     p_register=0.01, p_ack=0.01)
    raw, off = gen_payloads(spec, 4000, 1_700_000_000_000, seed=5)
    raw = np.concatenate([raw, np.zeros(64, np.uint8)])
    parts = (8, 4, 8, 2)
    for b in range(2):                      # the second step replays the batch: all duplicates dropped
        rg = g.step(raw, off, 1_700_000_001_000 + b, presence=False)
        rc = c.step(raw, off, 1_700_000_001_000 + b, presence=False)
        assert rg.n_persisted == rc.n_persisted
        cnt, _ = g.reject_refs_async(0, g._stg[2], g._stg[3], len(off) - 1)
        torch.cuda.synchronize()
        hdr = cnt.cpu().numpy().view(np.uint32)
        refs, comp = g.reject_snapshot(0, int(hdr[0]), int(hdr[1]))
        refs, comp = refs.copy(), comp.copy()
        gpu = routing.route_refs(comp, refs, 0, "gpu-inbound", parts)
        host = routing.route_rejects(raw, off, rc.rejects["aux_off"], rc.reject_status, "gpu-inbound", parts)
        assert len(gpu) > 0 and gpu.payloads == host.payloads
        gk = sorted((k, p, bytes(kh), bytes(vh)) for k, p, kh, ko, vh, vo in gpu.groups())
        hk = sorted((k, p, bytes(kh), bytes(vh)) for k, p, kh, ko, vh, vo in host.groups())
        assert gk == hk
