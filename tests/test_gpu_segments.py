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


def _encode_gpu(rows, recs, spans, raw, c0=0, seed=0):
    """Run k_seg_encode on one step's inputs laid out as the engine lays them out: device events in a
    permuted work array reached through ok_idx, generated rows after them, strings in the raw batch;
    the encoder aux rows built from them by ``k_seg_aux`` (the persist kernel's per-row write)."""
    import torch
    from sitewhere_amd._native import gpu
    from sitewhere_amd.models.columnar import EVENT_REC, OUT_REC, STR_REF
    from sitewhere_amd.persistence.segments import PAGE_ROWS, max_block_bytes, max_string_bytes
    lib = gpu()
    n = len(rows)
    d = torch.device("cuda", 0)
    dev = (recs["fp_lo"] != 0) | (recs["fp_hi"] != 0)
    n_ok = int(dev.sum())
    assert dev[:n_ok].all()                                  # device events first, generated after
    perm = np.random.default_rng(seed).permutation(n_ok)     # work position of persisted row j
    work = np.zeros(max(n_ok, 1), EVENT_REC)
    wsp = np.zeros(max(n_ok, 1), STR_REF)
    work[perm] = recs[:n_ok]
    wsp[perm] = spans[:n_ok]
    gen = np.ascontiguousarray(recs[n_ok:]) if n > n_ok else np.zeros(1, EVENT_REC)

    def t(a):
        return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).to(d)
    max_rows = max(n, 1) + 3000
    out_rows = torch.zeros(max_rows * OUT_REC.itemsize, dtype=torch.uint8, device=d)
    if n:
        out_rows[:n * OUT_REC.itemsize] = t(np.ascontiguousarray(rows, OUT_REC))
    work_t, wsp_t, gen_t = t(work), t(wsp), t(gen)
    okidx = torch.from_numpy(perm.astype(np.int32) if n_ok else np.zeros(1, np.int32)).to(d)
    nok = torch.tensor([n_ok], dtype=torch.int32, device=d)
    raw_t = t(np.concatenate([raw, np.zeros(64, np.uint8)]))
    cursor = torch.tensor([c0 + n, c0], dtype=torch.int64, device=d)
    bcap = max_block_bytes(max_rows, max_string_bytes(max_rows, len(raw)))
    pages = -(-max_rows // PAGE_ROWS)
    blk = torch.zeros(bcap, dtype=torch.uint8, device=d)
    state = torch.zeros(pages + 8, dtype=torch.int64, device=d)
    s = torch.cuda.current_stream(d)
    P = ctypes.c_void_p
    # encoder aux rows from the records (what the engine's persist kernel writes beside each row)
    aux = torch.zeros(max_rows * 32, dtype=torch.uint8, device=d)
    rc = lib.sw_seg_aux(P(work_t.data_ptr()), P(okidx.data_ptr()), P(nok.data_ptr()), P(gen_t.data_ptr()),
                        P(wsp_t.data_ptr()), len(raw), P(cursor.data_ptr()), P(aux.data_ptr()), max_rows,
                        P(s.cuda_stream))
    assert rc == 0
    rc = lib.sw_seg_encode(P(out_rows.data_ptr()), P(aux.data_ptr()), P(raw_t.data_ptr()), P(cursor.data_ptr()),
                           P(blk.data_ptr()), bcap, P(state.data_ptr()), pages, P(s.cuda_stream))
    assert rc == 0
    s.synchronize()
    nb, err, first = (int(x) for x in state[pages + 1:pages + 4].cpu().numpy())
    assert err == 0 and 0 < nb <= bcap, (nb, err)
    assert first == c0
    return blk[:nb].cpu().numpy()


def _same_bytes(g, c):
    assert len(g) == len(c), (len(g), len(c))
    if not np.array_equal(g, c):
        bad = np.nonzero(g != c)[0]
        pytest.fail(f"{len(bad)} bytes differ, first at {bad[0]} of {len(c)}")


@pytest.mark.parametrize("n,c0,full", [(0, 0, False), (1, 0, False), (1023, 0, False), (1024, 0, False),
                                       (1025, 5, False), (70_000, 0, True), (70_000, 60_000, False),
                                       (2_000_000, 0, False)])
def test_gpu_block_matches_cpu(n, c0, full):
    from sitewhere_amd.persistence import segments as sg
    from tests.test_segments import synth_rows
    rows, recs, spans, raw = synth_rows(n, seed=n + c0, full_precision=full)
    g = _encode_gpu(rows, recs, spans, raw, c0=c0, seed=n)
    c = sg.encode_block(rows, recs, spans, raw)
    _same_bytes(g, c)
    sg.seal(g, c0, 1, 2, 0, 1)
    assert sg.verify(g) == 0


def test_gpu_block_every_string_form_matches_cpu():
    """Raw- and hex-mode pages, multi-measurement suffixes, messages, metadata, updateState and
    elevation flags, and strings straddling heap words: GPU block == CPU block byte for byte."""
    from sitewhere_amd.models import wire
    from sitewhere_amd.models.columnar import EV_LOCATION, NO_NAME, OUT_REC
    from sitewhere_amd.persistence import segments as sg
    from sitewhere_amd.pipeline.fleet import cpu_decode, pack_messages
    msgs = []
    for i in range(6000):
        md = {f"k{j}": "v" * (i % 23) for j in range(i % 4)}
        alt = [f"{i:08x}", f"uuid-{i * 7919 % 104729}-{'y' * (i % 9)}", None, f"dev-9-{i}"][(i // 1500) % 4]
        k = i % 5
        if k == 0:
            msgs.append(wire.measurements(f"d-{i}", {"t": i / 100, "h": -i / 10}, alternate_id=alt, metadata=md,
                                          update_state=[None, True, False][i % 3]))
        elif k == 1:
            msgs.append(wire.location(f"d-{i}", 33 + i / 1e6, -84 - i / 1e6, elevation=None if i % 2 else i / 10,
                                      alternate_id=alt, metadata=md))
        elif k == 2:
            msgs.append(wire.alert(f"d-{i}", f"type{i % 7}", f"alert number {i}" * (1 + i % 3), alternate_id=alt,
                                   metadata=md))
        else:
            msgs.append(wire.measurements(f"d-{i}", {"only": float(i)}, alternate_id=alt))
    raw, offs = pack_messages(msgs)
    raw = raw[:int(offs[-1])]
    recs, spans = cpu_decode(raw, offs, 1_700_000_000_000, cap=16000, spans=True)
    rows = np.zeros(len(recs), OUT_REC)
    for k in ("event_date", "v0", "v1", "etype", "level"):
        rows[k] = recs[k]
    rows["assignment"] = np.arange(len(recs)) % 77
    rows["name_id"] = np.where(recs["etype"] == EV_LOCATION, NO_NAME, 3)
    g = _encode_gpu(rows, recs, spans, raw, seed=3)
    c = sg.encode_block(rows, recs, spans, raw)
    _same_bytes(g, c)
    cols = sg.decode_block(c, check=False)            # not sealed: no header checksum yet
    assert {int(f) & sg.SEGF_HAS_META for f in cols["flags"]} == {0, sg.SEGF_HAS_META}


def _decoded_equal(cg, cc, what):
    """Two decoded blocks hold the same events (name ids aside: engine-local, compared by name)."""
    # name ids are engine-local, so page sizes (and the header checksum over the page table) may differ
    strip = lambda h: {k: v for k, v in h.items() if k not in ("checksum", "bytes")}  # noqa: E731
    assert strip(cg["header"]) == strip(cc["header"]), what
    for k in ("etype", "level", "date", "asg", "v0", "v1", "v2", "flags", "str_off"):
        np.testing.assert_array_equal(cg[k], cc[k], err_msg=f"{what}: column {k}")
    end = int(cc["str_off"][-1]) if cc["str_off"] is not None and len(cc["str_off"]) else 0
    assert np.array_equal(cg["str_heap"][:end], cc["str_heap"][:end]), what


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
                     mx_per_msg=2, with_alternate_id=True, lat0=32.8, lon0=-85.2, span_deg=1.5, p_meta=0.2)
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
        _decoded_equal(cg, cc, f"step {b}")
        assert sum(sg.row_strings(cc, i)[0] is not None for i in range(len(cc["date"]))) > 1000
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
