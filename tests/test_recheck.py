"""Store-backed dedup of re-keyed records (``pipeline/recheck.py``): string compaction, the ids the
store is asked about, and re-injection into the oracle's re-key carry."""
from __future__ import annotations

import numpy as np

from sitewhere_amd.models.columnar import (EV_ALERT, EV_MEASUREMENT, EVENT_REC, F_SETTLED, SR_ALT, SR_META,
                                           SR_MULTI, STR_REF)
from sitewhere_amd.pipeline.recheck import alternate_ids, compact_strings, rebase_into


def _records():
    heap = bytearray(b"..........")
    recs = np.zeros(4, EVENT_REC)
    spans = np.zeros(4, STR_REF)

    def put(b):
        off = len(heap)
        heap.extend(b)
        return off, len(b)
    # 0: measurement with an id and metadata; 1: second measurement of a multi-measurement payload
    # (id "<alt>:1"); 2: alert with id and message; 3: control record (no strings travel)
    recs["etype"] = [EV_MEASUREMENT, EV_MEASUREMENT, EV_ALERT, 20]
    a0, l0 = put(b"alt-zero")
    m0, ml0 = put(b"\x22\x04name")
    spans[0] = (a0, m0, l0, ml0, 0, SR_ALT | SR_META, 0)
    a1, l1 = put(b"alt-multi")
    spans[1] = (a1, 0, l1, 0, 1, SR_ALT | SR_MULTI, 0)
    a2, l2 = put(b"alt-alert")
    g2, gl2 = put(b"door open")
    spans[2] = (a2, 0, l2, 0, 0, SR_ALT, 0)
    recs["aux2_off"][2], recs["aux2_len"][2] = g2, gl2
    recs["aux2_off"][3], recs["aux2_len"][3] = 1234, 9           # a control record's raw offsets stay
    return recs, spans, np.frombuffer(bytes(heap), np.uint8)


def test_compact_strings_layout_and_ids():
    recs, spans, heap = _records()
    r, s, h = compact_strings(recs, spans, lambda pos: heap[pos])
    # back to back: alt + meta, alt, alt + message, nothing for the control record
    assert bytes(h) == b"alt-zero\x22\x04name" + b"alt-multi" + b"alt-alert" + b"door open"
    assert (s["alt_off"][0], s["meta_off"][0], s["alt_len"][0], s["meta_len"][0]) == (0, 8, 8, 6)
    assert (s["alt_off"][1], s["alt_len"][1], s["k"][1], s["has"][1]) == (14, 9, 1, SR_ALT | SR_MULTI)
    assert (r["aux2_off"][2], r["aux2_len"][2]) == (32, 9)
    assert s["has"][3] == 0 and (r["aux2_off"][3], r["aux2_len"][3]) == (1234, 9)
    assert alternate_ids(s, h) == ["alt-zero", "alt-multi:1", "alt-alert", None]


def test_rebase_into_a_larger_heap():
    recs, spans, heap = _records()
    r, s, h = compact_strings(recs, spans, lambda pos: heap[pos])
    r2, s2 = rebase_into(r, s, 100, F_SETTLED)
    assert (r2["flags"] & F_SETTLED).all()
    assert s2["alt_off"][0] == 100 and s2["meta_off"][0] == 108 and r2["aux2_off"][2] == 132
    assert r2["aux2_off"][3] == 1234                               # control record untouched
    big = np.concatenate([np.zeros(100, np.uint8), h])
    assert alternate_ids(s2, big) == ["alt-zero", "alt-multi:1", "alt-alert", None]


def test_inject_settled_appends_to_the_oracle_carry():
    from sitewhere_amd.pipeline.config import EngineConfig
    from sitewhere_amd.pipeline.cpu_engine import CpuInboundEngine
    e = CpuInboundEngine(EngineConfig.small(world=2, rank=0))
    recs, spans, heap = _records()
    r, s, h = compact_strings(recs[:3], spans[:3], lambda pos: heap[pos])
    e.inject_settled(r, s, h)
    e.inject_settled(r[:1], s[:1], h[:14])
    assert len(e.carry) == 4 and len(e.carry_sp) == 4 and len(e.carry_heap) == len(h) + 14
    assert (e.carry["flags"] & F_SETTLED).all()
    assert alternate_ids(e.carry_sp, e.carry_heap) == ["alt-zero", "alt-multi:1", "alt-alert", "alt-zero"]
    st = e.checkpoint_state()
    e2 = CpuInboundEngine(EngineConfig.small(world=2, rank=0))
    e2.restore_state(st, include_store=False)
    assert np.array_equal(e2.carry_heap, e.carry_heap) and np.array_equal(e2.carry_sp, e.carry_sp)


def _packages(recs, spans, heap):
    """Recheck packages as ``k_reject_refs`` writes them (csrc/hip/swgpu.hip): record, string ref
    (offsets relative to the strings), strings; refs (0, bytes, status | src << 8 | packed, at)."""
    from sitewhere_amd.pipeline.recheck import REF_PACKED
    r, s, h = compact_strings(recs, spans, lambda pos: heap[pos])
    buf, refs = bytearray(b"pad"), []
    for i in range(len(r)):
        al, ml = int(s["alt_len"][i]), int(s["meta_len"][i])
        gl = int(r["aux2_len"][i]) if r["etype"][i] == EV_ALERT else 0
        base = int(s["alt_off"][i])
        one_r, one_s = r[i:i + 1].copy(), s[i:i + 1].copy()
        if al + ml + gl:
            one_s["alt_off"], one_s["meta_off"] = 0, al
            if gl:
                one_r["aux2_off"] = al + ml
        strings = bytes(h[base:base + al + ml + gl])
        at = len(buf)
        buf += one_r.tobytes() + one_s.tobytes() + strings
        refs.append((0, 96 + len(strings), 6 | (1 << 8) | REF_PACKED, at))
    refs.append((5, 9, 1, 0))                                    # an unregistered payload's ref
    refs.append((0, 120, 6 | REF_PACKED, 0xFFFFFFFF))             # a package that did not fit
    return np.array(refs, np.uint32), np.frombuffer(bytes(buf), np.uint8)


def test_unpack_rechecks_and_settle_later():
    """The owner reads rechecks from a reject snapshot's packages (several ranks, bench.py's
    pipelined path) and settles them: held ids are duplicates, the rest are handed to a deferred
    injector (re-injected between rounds)."""
    from sitewhere_amd.pipeline.recheck import settle, unpack_rechecks
    recs, spans, heap = _records()
    refs, comp = _packages(recs[:3], spans[:3], heap)
    r, s, h, lost = unpack_rechecks(refs, comp)
    assert lost == 1 and len(r) == 3
    assert alternate_ids(s, h) == ["alt-zero", "alt-multi:1", "alt-alert"]
    assert bytes(h[int(r["aux2_off"][2]):int(r["aux2_off"][2]) + 9]) == b"door open"
    assert bytes(h[int(s["meta_off"][0]):int(s["meta_off"][0]) + 6]) == b"\x22\x04name"
    r["alt_hash"] = [11, 22, 33]
    later = []
    c = settle(None, r, s, h, lambda hs: [int(x) == 22 for x in hs], by_hash=True,
               inject=lambda *x: later.append(x))
    assert c == {"rechecks": 3, "duplicates": 1, "injected": 2}
    (ir, isp, ih), = later
    assert list(ir["alt_hash"]) == [11, 33] and alternate_ids(isp, ih) == ["alt-zero", "alt-alert"]
