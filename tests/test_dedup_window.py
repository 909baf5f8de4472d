"""Generational alternate-id dedup window (reference AlternateIdDeduplicator.java:41-56).

Pushes far more distinct alternate ids than the window holds (several generations) through the
Python oracle and the native engine -- and the MI355X engine when present -- with replays of recent
batches (inside the window: duplicates) and of old ones (retired generations: new again).  All
engines must agree event for event, the window must actually rotate, and nothing may overflow
silently (``dedup_overflow`` stays 0)."""
from __future__ import annotations

import numpy as np
import pytest

from sitewhere_amd.pipeline.config import EngineConfig
from sitewhere_amd.pipeline.cpu_engine import CpuInboundEngine
from sitewhere_amd.pipeline.fleet import FleetSpec, fingerprints, gen_payloads, gen_tokens
from sitewhere_amd.pipeline.native_engine import NativeCpuEngine
from tests.conftest import gpu_available

CFG = dict(max_msgs=1024, gen_cap=1024, max_devices=2048, max_assignments=2048, store_cap=1 << 15,
           dedup_slots=1 << 12, name_slots=1 << 10, names_cap=1024)
N_DEV = 1500


def _split(raw, offs):
    return [bytes(raw[offs[i]:offs[i + 1]]) for i in range(len(offs) - 1)]


def _batches(n_batches=40, per=300):
    """Fresh batches (unique ids) with replays of the previous batch and of one 20 batches back."""
    spec = FleetSpec(prefix="dev-", n_devices=N_DEV, with_alternate_id=True, mx_per_msg=1, p_location=0.2,
                     p_alert=0.05)
    fresh = []
    for b in range(n_batches):
        raw, offs = gen_payloads(spec, per, 1_700_000_000_000 + 1000 * b, seed=100 + b)
        fresh.append(_split(raw, offs))
    out = []
    for b in range(n_batches):
        msgs = list(fresh[b])
        if b >= 1:
            msgs += fresh[b - 1][:40]          # recent replay: inside the window
        if b >= 20:
            msgs += fresh[b - 20][:40]         # late replay: long retired
        out.append(msgs)
    return out


def _engines():
    es = [CpuInboundEngine(EngineConfig.small(**CFG)), NativeCpuEngine(EngineConfig.small(**CFG))]
    if gpu_available():
        from sitewhere_amd.pipeline.gpu_engine import GpuInboundEngine
        es.append(GpuInboundEngine(EngineConfig.small(**CFG), device="cuda:0"))
    heap, offs = gen_tokens("dev-", 0, N_DEV)
    lo, hi = fingerprints(heap, offs)
    for e in es:
        d = e.register_devices(lo, hi)
        e.set_assignments(d, d)
    return es


def _run(engines):
    from sitewhere_amd.pipeline.fleet import pack_messages
    per_step = []
    for b, msgs in enumerate(_batches()):
        raw, offs = pack_messages(msgs)
        res = [e.step(raw, offs, 1_700_000_100_000 + b, presence=False) for e in engines]
        per_step.append([(r.n_persisted, int(np.sum(r.reject_status == 3))) for r in res])
    return per_step


def _check(engines, per_step):
    for b, row in enumerate(per_step):
        assert all(x == row[0] for x in row), f"batch {b}: engines disagree {row}"
    stats = [e.stats_dict() for e in engines]
    for s in stats[1:]:
        assert s == stats[0], (stats[0], s)
    s = stats[0]
    assert s["dedup_rotations"] >= 4            # ~12K distinct ids through a 2K-id generation
    assert s["dedup_overflow"] == 0
    # recent replays are always duplicates; replays 20 batches late (3+ generations) are not
    dups = [row[0][1] for row in per_step]
    assert all(d >= 40 for d in dups[1:20])
    assert all(40 <= d < 80 for d in dups[20:]), dups[20:]


def test_dedup_window_host_engines_agree():
    engines = _engines()[:2]
    _check(engines, _run(engines))


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
def test_dedup_window_gpu_matches_oracle():
    engines = _engines()
    assert len(engines) == 3
    _check(engines, _run(engines))


# ---------------------------------------------------------------------------- store-backed filter
# generational fingerprint tables (pipeline/dedup_filter.py): 4 generations of 4096 ids hold the
# newest >= 12288 ids of the run (~13K fresh ids + replays)
FCFG = dict(CFG, dedup_filter_ids=4096, dedup_filter_gens=4)


def _engines_filter(**kw):
    cfg = dict(FCFG, **kw)
    es = [CpuInboundEngine(EngineConfig.small(**cfg)), NativeCpuEngine(EngineConfig.small(**cfg))]
    if gpu_available():
        from sitewhere_amd.pipeline.gpu_engine import GpuInboundEngine
        es.append(GpuInboundEngine(EngineConfig.small(**cfg), device="cuda:0"))
    heap, offs = gen_tokens("dev-", 0, N_DEV)
    lo, hi = fingerprints(heap, offs)
    for e in es:
        d = e.register_devices(lo, hi)
        e.set_assignments(d, d)
    return es


def _run_filter(engines, batches=None):
    from sitewhere_amd.models.columnar import ST_RECHECK
    from sitewhere_amd.pipeline.fleet import pack_messages
    per_step = []
    for b, msgs in enumerate(batches if batches is not None else _batches()):
        raw, offs = pack_messages(msgs)
        res = [e.step(raw, offs, 1_700_000_100_000 + b, presence=False) for e in engines]
        per_step.append([(r.n_persisted, int(np.sum(r.reject_status == 3)), int(np.sum(r.reject_status == ST_RECHECK)),
                          sorted(r.rejects["alt_hash"][r.reject_status == ST_RECHECK].tolist())) for r in res])
    return per_step


def _check_filter(engines, per_step):
    for b, row in enumerate(per_step):
        assert all(x == row[0] for x in row), f"batch {b}: engines disagree"
    stats = [e.stats_dict() for e in engines]
    for s in stats[1:]:
        assert s == stats[0], (stats[0], s)
    fs = [e.filter_state() for e in engines]
    for f in fs[1:]:
        assert f == fs[0], (fs[0], f)
    s = stats[0]
    assert s["dedup_rotations"] >= 4 and s["dedup_overflow"] == 0
    assert fs[0]["rotations"] >= 2 and fs[0]["dropped"] == 0
    # recent replays: duplicates inside the window; late replays (retired window generations, still
    # in the filter): every one is handed to the host for a store check instead of being stored twice
    for b, row in enumerate(per_step):
        _, dups, rechecks, _ = row[0]
        assert dups >= 40 if b >= 1 else dups == 0
        assert rechecks == (40 if b >= 20 else 0), (b, rechecks)        # no false positive at all


def test_store_backed_filter_host_engines_agree():
    engines = _engines_filter()[:2]
    _check_filter(engines, _run_filter(engines))


def _batches_long(n_batches=80, per=300):
    """Fresh batches with replays 20 batches back (6000 ids: past the window, held by the filter) and
    60 back (18000 ids: older than any generation the filter keeps -- forgotten, as retention by rows
    has dropped them from a store sized to the filter)."""
    spec = FleetSpec(prefix="dev-", n_devices=N_DEV, with_alternate_id=True, mx_per_msg=1, p_location=0.2,
                     p_alert=0.05)
    fresh = []
    for b in range(n_batches):
        raw, offs = gen_payloads(spec, per, 1_700_000_000_000 + 1000 * b, seed=500 + b)
        fresh.append(_split(raw, offs))
    out = []
    for b in range(n_batches):
        msgs = list(fresh[b])
        if b >= 20:
            msgs += fresh[b - 20][:40]
        if b >= 60:
            msgs += fresh[b - 60][:30]
        out.append(msgs)
    return out


def _check_rotation_past_retention(engines, per_step):
    for b, row in enumerate(per_step):
        assert all(x == row[0] for x in row), f"batch {b}: engines disagree"
    fs = [e.filter_state() for e in engines]
    for f in fs[1:]:
        assert f == fs[0], (fs[0], f)
    assert fs[0]["rotations"] >= 4 and fs[0]["dropped"] == 0        # the filter wrapped past every generation
    for b, row in enumerate(per_step):
        persisted, dups, rechecks, _ = row[0]
        assert dups == 0, (b, dups)
        # the 20-back replays are rechecked; the 60-back ones are new to the filter again (persisted)
        assert rechecks == (40 if b >= 20 else 0), (b, rechecks)
        if b >= 60:
            assert persisted == 300 + 30, (b, persisted)


def test_store_backed_filter_rotates_past_retention():
    engines = _engines_filter()[:2]
    _check_rotation_past_retention(engines, _run_filter(engines, _batches_long()))


def test_store_backed_filter_warm_start_and_checkpoint():
    """The filter travels in engine checkpoints and can be seeded from stored ids (``filter_seed``,
    newest first -- what a restarted tenant does from its durable store): ids seeded that way are
    rechecked, and a seed larger than the filter keeps only the newest."""
    from sitewhere_amd.models.columnar import ST_RECHECK
    from sitewhere_amd.pipeline.fleet import pack_messages
    raw, offs = pack_messages(_batches(n_batches=1)[0][:300])
    for idx in (0, 1):                                 # oracle, native engine
        a = _engines_filter()[idx]
        a.step(raw, offs, 1_700_000_100_000, presence=False)
        ck = a.checkpoint_state()
        assert "dd_ff_idx" in ck and len(ck["dd_ff_idx"]) > 0 and np.asarray(ck["dd_ff_rows"]).any()
        b = _engines_filter()[idx]
        b.restore_state(ck, include_store=False)
        ck2 = b.checkpoint_state()
        assert np.array_equal(ck2["dd_ff_idx"], ck["dd_ff_idx"]) and np.array_equal(ck2["dd_ff_rows"], ck["dd_ff_rows"])
        assert b.filter_state() == a.filter_state()
        c = _engines_filter()[idx]
        c.filter_seed_begin()
        assert c.filter_seed(_alt_hashes(raw, offs)) == len(_alt_hashes(raw, offs))
        r = c.step(raw, offs, 1_700_000_300_000, presence=False)
        assert int(np.sum(r.reject_status == ST_RECHECK)) == len(_alt_hashes(raw, offs)), idx
        # 5 generations' worth, newest first: the 4 newest generations' ids are kept, the oldest not
        d = _engines_filter(dedup_filter_ids=4096, dedup_filter_gens=2)[idx]
        ids = np.arange(1, 3 * 4096 + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
        d.filter_seed_begin()
        assert d.filter_seed(ids[:5000]) + d.filter_seed(ids[5000:]) == 2 * 4096
        st = d.filter_state()
        assert st["live_ids"] == 4096
        have = [d.ff.has(int(h)) if idx == 0 else None for h in ids[[0, 4095, 4096, 8191, 8192, 12287]]]
        if idx == 0:
            assert have == [True, True, True, True, False, False]


def _alt_hashes(raw, offs):
    from sitewhere_amd.pipeline.fleet import cpu_decode
    recs = cpu_decode(raw, offs, 1_700_000_000_000)
    return recs["alt_hash"][recs["alt_hash"] != 0]


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
def test_store_backed_filter_gpu_matches_oracle():
    engines = _engines_filter()
    assert len(engines) == 3
    _check_filter(engines, _run_filter(engines))


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
def test_store_backed_filter_gpu_rotates_past_retention():
    engines = _engines_filter()
    assert len(engines) == 3
    _check_rotation_past_retention(engines, _run_filter(engines, _batches_long()))
