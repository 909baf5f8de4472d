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
