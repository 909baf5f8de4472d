"""Bench-scale parity: the MI355X engine against the native CPU engine (bit-exact
with the Python oracle) in the configuration bench.py runs -- 1M-payload steps over a 1M-device fleet
with alternate ids, metadata and control messages, a 2^22-slot dedup window that rotates several
times, the store-backed alternate-id filter (generational fingerprint tables), an HBM event ring that wraps
every two steps, and replays inside and beyond the window.  Every step: same stats, same persisted
rows (device events in order, generated rows as a multiset), same reject statuses, the same durable
block contents and the same block index trailer (built on the GPU in the step vs by the C++
builder on the CPU engine's block).  The replay beyond the window comes back as rechecks (the
filter remembers the ids), not as accepted events.  A second run rotates the filter itself past
everything it holds: replays it still holds are rechecked, older ones are new again,
and the two engines agree on every step and on the filter's state."""
from __future__ import annotations

import numpy as np
import pytest

from tests.conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs an MI355X GPU")]

N_MSGS = 1 << 20
N_DEV = 1 << 20


def _cfg(**kw):
    from sitewhere_amd.pipeline.config import EngineConfig
    base = dict(max_msgs=N_MSGS, rec_cap=N_MSGS + 4096, gen_cap=N_MSGS // 2, max_devices=N_DEV + 1024,
                max_assignments=N_DEV + 1024, store_cap=1 << 21, dedup_slots=1 << 22, name_slots=1 << 12,
                state_slots=1 << 23, presence_missing_ms=8 * 3600 * 1000, dedup_filter_ids=1 << 26,
                dedup_filter_gens=4)
    base.update(kw)
    return EngineConfig(**base)


def _setup(engine):
    from sitewhere_amd.pipeline.engine_base import Zone, ZoneTest
    from sitewhere_amd.pipeline.fleet import fingerprints, gen_tokens
    heap, offs = gen_tokens("dev-", 0, N_DEV)
    lo, hi = fingerprints(heap, offs)
    dev = engine.register_devices(lo, hi)
    engine.set_assignments(dev, dev, customer=dev % 97, area=dev % 31, asset=dev % 1009)
    sq = [(33.0, -85.0), (33.0, -84.0), (34.0, -84.0), (34.0, -85.0)]
    engine.set_zone_rules([Zone("z", sq)], [ZoneTest("z", "inside", "zone.enter", 2)])


def _rows_equal(rg, rc, name_g, name_c, dev):
    """Device rows (the first ``dev``) in order, generated rows as a multiset; name ids compared
    through the names they stand for."""
    og, oc = rg.out, rc.out
    assert len(og) == len(oc)
    ng = name_g(og["name_id"])
    nc = name_c(oc["name_id"])
    keys = ("etype", "assignment", "event_date", "v0", "v1", "level")
    cols_g = np.stack([og[k].astype(np.float64) for k in keys] + [ng.astype(np.float64)], 1)
    cols_c = np.stack([oc[k].astype(np.float64) for k in keys] + [nc.astype(np.float64)], 1)
    assert np.array_equal(cols_g[:dev], cols_c[:dev])
    sg = cols_g[np.lexsort(cols_g.T[::-1])]
    sc = cols_c[np.lexsort(cols_c.T[::-1])]
    assert np.array_equal(sg, sc)


def _name_map(engine):
    inv = {i: h for h, i in engine.intern_table().items()}
    table = np.zeros(1 << 16, np.uint64)
    for i, h in inv.items():
        if 0 <= i < len(table):
            table[i] = np.uint64(h)
    table[0xFFFF] = 0
    return lambda ids: table[np.asarray(ids, np.int64)]


def test_gpu_matches_native_cpu_engine_at_bench_scale():
    import torch  # noqa: F401
    from sitewhere_amd.persistence import segments as sg
    from sitewhere_amd.pipeline.fleet import FleetSpec, gen_payloads
    from sitewhere_amd.pipeline.gpu_engine import GpuInboundEngine
    from sitewhere_amd.pipeline.native_engine import NativeCpuEngine
    g = GpuInboundEngine(_cfg(), device="cuda:0")
    c = NativeCpuEngine(_cfg(), threads=16)
    for e in (g, c):
        _setup(e)
    spec = FleetSpec(prefix="dev-", n_devices=N_DEV, p_location=0.25, p_alert=0.05, p_unregistered=0.005,
                     mx_per_msg=1, n_names=16, with_alternate_id=True, lat0=33.0, lon0=-85.0, span_deg=2.0,
                     p_register=0.0005, p_ack=0.0005, p_meta=0.1)
    now = 1_700_000_100_000
    # 1..6 fresh; 5 again (inside the window: all duplicates); 7..9 fresh (the window rotates: 2^22
    # slots hold 2M-4M ids); 1 again (beyond the window: the filter sends every id to a recheck)
    seeds = [1, 2, 3, 4, 5, 6, 5, 7, 8, 9, 1]
    batches = {}
    dups, rechecks = [], []
    for k, seed in enumerate(seeds):
        if seed not in batches:
            raw, offs = gen_payloads(spec, N_MSGS, now - 60_000, seed=seed)
            batches[seed] = (np.concatenate([raw, np.zeros(64, np.uint8)]), offs)
        raw, offs = batches[seed]
        s0 = g.stats_dict()
        rg = g.step(raw, offs, now + k, presence=(k % 4 == 3))
        rc = c.step(raw, offs, now + k, presence=(k % 4 == 3))
        assert g.stats_dict() == c.stats_dict(), f"step {k}"
        dups.append(g.stats_dict()["duplicates"] - s0["duplicates"])
        rechecks.append(g.stats_dict()["dedup_rechecks"] - s0["dedup_rechecks"])
        assert rg.n_persisted == rc.n_persisted
        # the replays: inside the window all duplicates, beyond it all rechecks
        assert rg.n_persisted > 0 or k in (6, 10)
        s1 = g.stats_dict()
        gen = (s1["rule_alerts"] - s0["rule_alerts"]) + (s1["presence_events"] - s0["presence_events"])
        _rows_equal(rg, rc, _name_map(g), _name_map(c), rg.n_persisted - gen)
        assert sorted(rg.reject_status.tolist()) == sorted(rc.reject_status.tolist())
        blk_g = g.encode_block(now + k, rg, boot=0xabc)
        blk_c = c.encode_block(now + k, rc, boot=0xabc)
        tg, tc = sg.trailer_offset(blk_g), sg.trailer_offset(blk_c)
        assert tg > 0 and tc > 0 and np.array_equal(blk_g[tg:], blk_c[tc:]), k       # index trailers
        bg, bc = sg.decode_block(blk_g), sg.decode_block(blk_c)
        for col in ("etype", "level", "date", "asg", "v0", "v1", "v2", "flags", "str_off"):
            assert np.array_equal(bg[col], bc[col]), (k, col)
        if bc["str_off"] is not None:
            end = int(bc["str_off"][-1])
            assert np.array_equal(bg["str_heap"][:end], bc["str_heap"][:end]), k
    st = g.stats_dict()
    assert st["dedup_rotations"] >= 2 and st["dedup_overflow"] == 0 and st["state_overflow"] == 0
    assert dups[6] > 0.99 * N_MSGS * (1 - spec.p_unregistered - 0.001)       # replay inside the window
    # replay beyond it: not accepted -- every id the filter has seen goes to the store recheck
    assert dups[10] == 0
    assert rechecks[10] > 0.99 * N_MSGS * (1 - spec.p_unregistered - 0.001)
    assert sum(rechecks[:6]) + sum(rechecks[7:10]) < 1000                    # the filter's false positives


def test_gpu_filter_rotates_past_retention_at_bench_scale():
    """2 generations of 2^22 ids: the filter holds the newest 4-9 batches' ids.  Replays 3 batches back
    (past the window, held) are all rechecks; replays 14 back (past every generation: what a store
    bounded by rows no longer holds) are new again.  GPU and native engine agree step by step."""
    from sitewhere_amd.pipeline.fleet import FleetSpec, gen_payloads
    from sitewhere_amd.pipeline.gpu_engine import GpuInboundEngine
    from sitewhere_amd.pipeline.native_engine import NativeCpuEngine
    kw = dict(dedup_filter_ids=1 << 22, dedup_filter_gens=2, state_slots=1 << 25)   # 16 steps of (asg, name) keys
    g = GpuInboundEngine(_cfg(**kw), device="cuda:0")
    c = NativeCpuEngine(_cfg(**kw), threads=16)
    for e in (g, c):
        _setup(e)
    spec = FleetSpec(prefix="dev-", n_devices=N_DEV, p_location=0.25, p_alert=0.05, p_unregistered=0.005,
                     mx_per_msg=1, n_names=16, with_alternate_id=True, lat0=33.0, lon0=-85.0, span_deg=2.0,
                     p_register=0.0005, p_ack=0.0005, p_meta=0.1)
    now = 1_700_000_200_000
    seeds = list(range(101, 115)) + [111, 101]
    batches, rechecks, dups, persisted = {}, [], [], []
    for k, seed in enumerate(seeds):
        if seed not in batches:
            raw, offs = gen_payloads(spec, N_MSGS, now - 60_000, seed=seed)
            batches[seed] = (np.concatenate([raw, np.zeros(64, np.uint8)]), offs)
        raw, offs = batches[seed]
        s0 = g.stats_dict()
        rg = g.step(raw, offs, now + k, presence=False)
        rc = c.step(raw, offs, now + k, presence=False)
        assert g.stats_dict() == c.stats_dict(), f"step {k}"
        assert g.filter_state() == c.filter_state(), f"step {k}"
        assert rg.n_persisted == rc.n_persisted
        s1 = g.stats_dict()
        rechecks.append(s1["dedup_rechecks"] - s0["dedup_rechecks"])
        dups.append(s1["duplicates"] - s0["duplicates"])
        persisted.append(rg.n_persisted)
    fs = g.filter_state()
    assert fs["rotations"] >= 2 and fs["dropped"] == 0
    valid = 0.99 * N_MSGS * (1 - spec.p_unregistered - 0.001)
    assert dups[14] == 0 and rechecks[14] > valid                       # held by the filter
    assert dups[15] == 0 and rechecks[15] == 0                           # forgotten: new again
    assert persisted[15] > valid
    assert sum(rechecks[:14]) == 0                                       # no false positive
