"""Store-backed dedup of re-keyed records (several ranks).

The reference asks the event store about every event's alternate id
(``AlternateIdDeduplicator.isDuplicate``, service-event-sources/.../AlternateIdDeduplicator.java:41-56).
Here an engine keeps the id window on the device and a blocked Bloom filter of every id it
persisted; an id new to the window that the filter may hold comes back as a *recheck*
(``ST_RECHECK``, not persisted).  On one rank the host re-reads the recheck's payload from the raw
batch (``services/gpu_inbound.py``).  On several ranks the record was decoded on another rank, but
the re-key brought its strings along (``SwEngineArgs.send_str``), so the owner settles it by its
alternate id:

  * :func:`settle_rechecks` asks the store (``held``) about each recheck's id string;
  * ids the store holds are duplicates (counted, dropped);
  * the rest -- filter false positives -- are re-injected into the engine's re-key carry with
    ``F_SETTLED`` (``engine.inject_settled``): the next round processes them like any record
    (window claim, state, rules, persistence) except that the filter skips them.

Strings travel in the layout the re-key's slabs and carry heap use (:func:`compact_strings`)."""
from __future__ import annotations

import numpy as np

from ..models.columnar import EV_ALERT, SR_ALT, SR_META, SR_MULTI, ST_RECHECK, STR_REF


def _excl(x: np.ndarray) -> np.ndarray:
    return np.cumsum(x) - x


def compact_strings(recs: np.ndarray, spans: np.ndarray, take):
    """Each record's alternate id, metadata and alert message copied back to back into one heap
    (the layout of the re-key's string slabs and carry heap).  ``take(positions)`` reads bytes of
    the source heap.  Returns (records with alert messages rebased, refs into the heap, heap)."""
    recs = np.array(recs, copy=True)
    n = len(recs)
    has = spans["has"].astype(np.int64)
    ctl = recs["etype"] >= 16
    al = np.where((has & SR_ALT) != 0, spans["alt_len"], 0).astype(np.int64)
    ml = np.where((has & SR_META) != 0, spans["meta_len"], 0).astype(np.int64)
    alert = recs["etype"] == EV_ALERT
    gl = np.where(alert, recs["aux2_len"], 0).astype(np.int64)
    al[ctl] = ml[ctl] = gl[ctl] = 0
    ln = al + ml + gl
    start = _excl(ln)
    total = int(ln.sum())
    src = np.zeros(total, np.int64)
    for off, lens, at in ((spans["alt_off"], al, start), (spans["meta_off"], ml, start + al),
                          (recs["aux2_off"], gl, start + al + ml)):
        m = lens > 0
        if not m.any():
            continue
        ll = lens[m]
        k = np.arange(int(ll.sum())) - np.repeat(_excl(ll), ll)
        src[np.repeat(at[m], ll) + k] = np.repeat(off[m].astype(np.int64), ll) + k
    heap = np.asarray(take(src), np.uint8) if total else np.zeros(0, np.uint8)
    ns = np.zeros(n, STR_REF)
    some = ~ctl & (ln > 0)
    ns["k"] = np.where(ctl, 0, spans["k"])
    ns["has"] = np.where(some, has, np.where(ctl, 0, has & SR_MULTI))
    ns["alt_off"] = np.where(some, start, 0)
    ns["meta_off"] = np.where(some, start + al, 0)
    ns["alt_len"] = al
    ns["meta_len"] = ml
    am = alert & ~ctl
    recs["aux2_off"] = np.where(am, np.where(gl > 0, start + al + ml, 0), recs["aux2_off"])
    recs["aux2_len"] = np.where(am, gl, recs["aux2_len"])
    return recs, ns, heap


def alternate_ids(spans: np.ndarray, heap: np.ndarray) -> list:
    """The alternate id each record is stored under ("<alt>", or "<alt>:<k>" for one measurement of
    a multi-measurement payload, as ``services/event_sources.py`` names them); None without one."""
    out = []
    for s in spans:
        if not int(s["has"]) & SR_ALT:
            out.append(None)
            continue
        o = int(s["alt_off"])
        a = bytes(heap[o:o + int(s["alt_len"])]).decode("utf-8", "replace")
        out.append(f"{a}:{int(s['k'])}" if int(s["has"]) & SR_MULTI else a)
    return out


def settle_rechecks(engine, res, held, by_hash: bool = False, inject=None) -> dict:
    """Settle the rechecks of one step result on the rank that owns them: ``held(ids)`` -> one bool
    per alternate id (the store holds it); ``by_hash``: ``held`` gets the ids' 64-bit hashes
    (``EVENT_REC["alt_hash"]``, what the durable store's alternate-id index answers) instead of the
    strings.  Held ids are duplicates; the rest are re-injected into the engine's carry,
    filter-settled -- or handed to ``inject(recs, spans, heap)`` when the caller re-injects them
    later (between pipelined rounds).  Returns counts."""
    rc = engine.rechecks(res)
    if rc is None:
        return {"rechecks": 0, "duplicates": 0, "injected": 0}
    return settle(engine, *rc, held, by_hash=by_hash, inject=inject)


def settle(engine, recs, spans, heap, held, by_hash: bool = False, inject=None) -> dict:
    """:func:`settle_rechecks` of rechecks already in the compact layout."""
    n = len(recs)
    keys = np.asarray(recs["alt_hash"], np.uint64) if by_hash else alternate_ids(spans, heap)
    dup = np.fromiter((bool(x) for x in held(keys)), bool, n) if n else np.zeros(0, bool)
    keep = ~dup
    if keep.any():
        (inject or engine.inject_settled)(*_select(recs, spans, heap, keep))
    return {"rechecks": n, "duplicates": int(dup.sum()), "injected": int(keep.sum())}


REF_PACKED = 0x10000       # k_reject_refs: the ref's copy is a recheck package, not a payload
_PKG_HDR = 80              # SwEventRec
_SREF = 16                 # SwStrRef


def unpack_rechecks(refs: np.ndarray, compact: np.ndarray):
    """The recheck packages of a reject snapshot (``k_reject_refs`` with strings exchanged: per
    recheck the 80-byte record, its string ref and its strings back to back) as (records, refs,
    heap) in the compact layout, plus the number of packages that did not fit the snapshot's byte
    buffer (those rechecks cannot be settled from it)."""
    from ..models.columnar import EVENT_REC, STR_REF
    refs = np.asarray(refs, np.uint32).reshape(-1, 4)
    pk = refs[(refs[:, 2] & REF_PACKED) != 0]
    have = pk[pk[:, 3] != 0xFFFFFFFF]
    lost = len(pk) - len(have)
    comp = np.asarray(compact, np.uint8)
    recs = np.zeros(len(have), EVENT_REC)
    spans = np.zeros(len(have), STR_REF)
    parts, base = [], 0
    for j, (_, ln, _, at) in enumerate(have.tolist()):
        blob = comp[at:at + ln]
        recs[j] = blob[:_PKG_HDR].view(EVENT_REC)[0]
        spans[j] = blob[_PKG_HDR:_PKG_HDR + _SREF].view(STR_REF)[0]
        s = blob[_PKG_HDR + _SREF:]
        if len(s):
            spans[j]["alt_off"] += base
            spans[j]["meta_off"] += base
            if recs[j]["etype"] == EV_ALERT and recs[j]["aux2_len"]:
                recs[j]["aux2_off"] += base
        parts.append(np.array(s, copy=True))
        base += len(s)
    heap = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
    return recs, spans, heap, lost


def _select(recs, spans, heap, mask):
    """The records of ``mask`` with their strings, re-compacted."""
    return compact_strings(recs[mask], spans[mask], lambda pos: heap[pos])


def host_rechecks(res):
    """Rechecks of a host engine's step result (records, refs, heap), None when there are none or
    the strings did not travel with the records (one rank: the payload path settles them)."""
    st = res.reject_status
    sp = getattr(res, "rspans", None)
    if st is None or sp is None or res.raw is None:
        return None
    rk = st == ST_RECHECK
    if not rk.any():
        return None
    src = np.asarray(res.raw, np.uint8)
    return compact_strings(res.rejects[rk], sp[rk], lambda pos: src[pos])


def rebase_into(recs: np.ndarray, spans: np.ndarray, base: int, flag: int):
    """Records / refs of a compact heap moved to offset ``base`` of a larger heap, ``flag`` set."""
    recs = np.array(recs, copy=True)
    spans = np.array(spans, copy=True)
    recs["flags"] |= np.uint8(flag)
    some = (spans["alt_len"].astype(np.int64) + spans["meta_len"]) > 0
    alert = (recs["etype"] == EV_ALERT) & (recs["aux2_len"] > 0)
    some |= alert
    spans["alt_off"] = np.where(some, spans["alt_off"].astype(np.int64) + base, spans["alt_off"])
    spans["meta_off"] = np.where(some, spans["meta_off"].astype(np.int64) + base, spans["meta_off"])
    recs["aux2_off"] = np.where(alert, recs["aux2_off"].astype(np.int64) + base, recs["aux2_off"])
    return recs, spans
