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
def _engines_bloom():
    cfg = dict(CFG, dedup_bloom_bits=1 << 20)           # 128 KB: ~87 bits per id of the run
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


def _run_bloom(engines):
    from sitewhere_amd.models.columnar import ST_RECHECK
    from sitewhere_amd.pipeline.fleet import pack_messages
    per_step = []
    for b, msgs in enumerate(_batches()):
        raw, offs = pack_messages(msgs)
        res = [e.step(raw, offs, 1_700_000_100_000 + b, presence=False) for e in engines]
        per_step.append([(r.n_persisted, int(np.sum(r.reject_status == 3)), int(np.sum(r.reject_status == ST_RECHECK)),
                          sorted(r.rejects["alt_hash"][r.reject_status == ST_RECHECK].tolist())) for r in res])
    return per_step


def _check_bloom(engines, per_step):
    for b, row in enumerate(per_step):
        assert all(x == row[0] for x in row), f"batch {b}: engines disagree"
    stats = [e.stats_dict() for e in engines]
    for s in stats[1:]:
        assert s == stats[0], (stats[0], s)
    s = stats[0]
    assert s["dedup_rotations"] >= 4 and s["dedup_overflow"] == 0
    # recent replays: duplicates inside the window; late replays (retired generations): every one is
    # handed to the host for a store check instead of being stored a second time
    for b, row in enumerate(per_step):
        _, dups, rechecks, _ = row[0]
        assert dups >= 40 if b >= 1 else dups == 0
        assert rechecks >= 40 if b >= 20 else True
    total_fresh = sum(300 for _ in per_step)
    assert s["dedup_rechecks"] - sum(40 for b in range(20, len(per_step))) < 0.01 * total_fresh   # false positives


def test_store_backed_filter_host_engines_agree():
    engines = _engines_bloom()[:2]
    _check_bloom(engines, _run_bloom(engines))


def test_store_backed_filter_warm_start_and_checkpoint():
    """The filter travels in engine checkpoints and can be seeded from stored ids (``bloom_add``, what
    a restarted tenant does from its store's alternate-id index): ids seeded that way are rechecked."""
    from sitewhere_amd.models.columnar import ST_RECHECK
    from sitewhere_amd.pipeline.fleet import pack_messages
    raw, offs = pack_messages(_batches(n_batches=1)[0][:300])
    for idx in (0, 1):                                 # oracle, native engine
        a = _engines_bloom()[idx]
        a.step(raw, offs, 1_700_000_100_000, presence=False)
        ck = a.checkpoint_state()
        assert "dd_bloom" in ck and np.asarray(ck["dd_bloom"]).any()
        b = _engines_bloom()[idx]
        b.restore_state(ck, include_store=False)
        assert np.array_equal(np.asarray(b.checkpoint_state()["dd_bloom"]), np.asarray(ck["dd_bloom"]))
        c = _engines_bloom()[idx]
        c.bloom_add(_alt_hashes(raw, offs))
        r = c.step(raw, offs, 1_700_000_300_000, presence=False)
        assert int(np.sum(r.reject_status == ST_RECHECK)) == len(_alt_hashes(raw, offs)), idx


def _alt_hashes(raw, offs):
    from sitewhere_amd.pipeline.fleet import cpu_decode
    recs = cpu_decode(raw, offs, 1_700_000_000_000)
    return recs["alt_hash"][recs["alt_hash"] != 0]


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")
def test_store_backed_filter_gpu_matches_oracle():
    engines = _engines_bloom()
    assert len(engines) == 3
    _check_bloom(engines, _run_bloom(engines))
