"""CPU implementation of the inbound pipeline (reference oracle + CPU fallback).

Implements exactly the stage semantics of ``csrc/hip/swgpu.hip`` with numpy and
the shared C++ decoder, one micro-batch at a time.  It is the parity oracle for
the GPU engine (tests/test_gpu_engine.py) and runs the multi-rank path over the
``gloo`` backend (tests/test_distributed_cpu.py), so the owner-partition +
all-to-all protocol is covered without GPUs.
"""
from __future__ import annotations

import numpy as np

from ..models.columnar import (EVENT_REC, OUT_REC, EV_ALERT, EV_LOCATION, EV_MEASUREMENT, EV_STATE_CHANGE,
                               EV_DECODE_ERROR, ST_OK, ST_UNREGISTERED, ST_UNASSIGNED, ST_DUPLICATE,
                               ST_DECODE_ERROR, ST_CONTROL, ST_RECHECK, STAT_NAMES, N_STATS, STR_REF, WIRE_REC,
                               F_SETTLED, wire_pack, wire_unpack)
from .config import EngineConfig
from .dedup_filter import FingerprintFilter
from .engine_base import EngineBase, StepResult
from .fleet import cpu_decode

_M64 = (1 << 64) - 1


def mix64(x: int) -> int:
    """sw_mix64 (csrc/include/swtypes.h)."""
    x &= _M64
    x ^= x >> 30
    x = (x * 0xbf58476d1ce4e5b9) & _M64
    x ^= x >> 27
    x = (x * 0x94d049bb133111eb) & _M64
    return x ^ (x >> 31)

STORE_COLS = {
    "etype": np.uint8, "level": np.uint8, "date": np.int64, "recv": np.int64, "dev": np.int32, "asg": np.int32,
    "cust": np.int32, "area": np.int32, "asset": np.int32, "name": np.uint64, "v0": np.float64, "v1": np.float64,
    "v2": np.float64, "alt": np.uint64, "aux": np.uint64, "batch": np.int32,
}


def pip(vtx: np.ndarray, x: float, y: float) -> bool:
    """Even-odd crossing-number point-in-polygon (same predicate as the kernel)."""
    inside = False
    n = len(vtx)
    j = n - 1
    for i in range(n):
        xi, yi = vtx[i]
        xj, yj = vtx[j]
        if ((yi > y) != (yj > y)) and (x < (xj - xi) * (y - yi) / (yj - yi) + xi):
            inside = not inside
        j = i
    return inside


class CpuInboundEngine(EngineBase):
    """Numpy engine shard; same interface as :class:`GpuInboundEngine`."""

    def __init__(self, cfg: EngineConfig, group=None):
        super().__init__(cfg)
        self.group = group
        self.exchange = None
        self.carry = np.zeros(0, EVENT_REC)    # records deferred to the next exchange (full slabs)
        # the carry's strings: refs into carry_heap (an alert's message offset is in its record)
        self.carry_sp = np.zeros(0, STR_REF)
        self.carry_heap = np.zeros(0, np.uint8)
        self.str_drops = [0, 0]                # [records sent without strings (larger than a slab), unused]
        self.store = {k: np.zeros(cfg.store_cap, t) for k, t in STORE_COLS.items()}
        self.cursor = 0
        self.seq_base = 0
        self.dedup: dict[int, int] = {}          # current generation of the alternate-id window
        self.dedup_prev: dict[int, int] = {}     # previous generation
        # store-backed dedup filter (generational fingerprint tables, pipeline/dedup_filter.py)
        self.ff = (FingerprintFilter(cfg.ff_buckets, cfg.dedup_filter_gens, cfg.dedup_filter_ids)
                   if cfg.dedup_filter_ids else None)
        self.intern: dict[int, int] = {}
        self.st_last = np.zeros(cfg.max_assignments, np.uint64)
        self.st_missing = np.zeros(cfg.max_assignments, np.uint64)
        self.st_loc_date = np.zeros(cfg.max_assignments, np.uint64)
        self.st_loc_eid = np.zeros(cfg.max_assignments, np.int64)   # eid + 1, 0 = none
        self.ms: dict[tuple, list] = {}                               # (asg, name_id, kind) -> [date, eid+1]
        self.stats = np.zeros(N_STATS, np.uint64)
        self._seen: set[int] = set()

    # ------------------------------------------------------------------ stages
    def partition(self, recs: np.ndarray, with_index: bool = False, spans=None, raw=None):
        """Stable owner partition into [world, shuf_cap] slabs (same as k_part_count / k_part_cut /
        k_part_write).

        The input is the previous partition's carry followed by ``recs``.  Per destination, records
        go to the slab in input order while they fit: a record slot (``shuf_cap``) and, with the
        string exchange on (``spans`` / ``raw`` given), its strings in the destination's byte slab
        (``str_cap``: the slab takes a prefix of the records, strings included).  The rest spill
        destination-major into the next carry (up to ``carry_cap``; beyond it, and beyond the carry's
        string heap, records are dropped and counted) -- with their strings, which the carry keeps
        (``carry_heap``), so a deferred record loses nothing.  A record whose strings alone exceed a
        slab is sent without them (``str_drops[0]``: impossible at the default sizes).
        ``with_index``: also the input indices of each slab's records and the carry length."""
        nc = len(self.carry)
        strings = spans is not None and raw is not None and bool(self.cfg.str_cap)
        inp = np.concatenate([self.carry, recs]) if nc else recs
        owner = self._dest(inp)
        cap, scap = self.cfg.shuf_cap, self.cfg.str_cap
        L = self._string_lengths(inp, nc, spans) if strings else np.zeros(len(inp), np.int64)
        over = L > scap if strings else np.zeros(len(inp), bool)
        if over.any():
            self.str_drops[0] += int(over.sum())
            L = np.where(over, 0, L)
        self._strip = over                      # records sent without their strings
        send = np.zeros((self.world, cap), EVENT_REC)
        cnt = np.zeros(self.world, np.int64)
        spill_idx = []
        index = []
        for o in range(self.world):
            at = np.nonzero(owner == o)[0]
            k = min(len(at), cap)
            if strings and k:
                k = int(np.searchsorted(np.cumsum(L[at[:k]]), scap, side="right"))
            send[o, :k] = inp[at[:k]]
            cnt[o] = k
            index.append(at[:k])
            spill_idx.append(at[k:])
        spill_idx = np.concatenate(spill_idx) if spill_idx else np.zeros(0, np.int64)
        kept = min(len(spill_idx), self.cfg.carry_cap)
        keep = spill_idx[:kept]
        if strings and kept:
            # the deferred records' strings move into the next carry's heap (up to its capacity)
            fits = np.cumsum(L[keep]) <= self.cfg.carry_str_cap
            if not fits.all():               # beyond the carry's string heap: dropped like beyond carry_cap
                kept = int(fits.sum())
                keep = keep[:kept]
        self.stats[13] += kept
        self.stats[10] += len(spill_idx) - kept
        old_sp, old_heap = self.carry_sp, self.carry_heap
        self._part_src = (nc, old_sp, old_heap)          # where _pack_strings reads carried strings
        new_carry = inp[keep].copy()
        if strings and kept:
            self.carry_sp, self.carry_heap = self._gather_strings(new_carry, keep, nc, spans, raw, old_sp, old_heap,
                                                                  L[keep], rebase_msg=True)
        else:
            self.carry_sp, self.carry_heap = np.zeros(kept, STR_REF), np.zeros(0, np.uint8)
        self.carry = new_carry
        if with_index:
            return send, cnt, index, nc
        return send, cnt

    def _string_lengths(self, inp, nc, spans) -> np.ndarray:
        """Exchange bytes of each partition input: alternate id + metadata + alert message (0 for
        control records); carried records' from the carry's refs."""
        n = len(inp)
        s = np.zeros(n, STR_REF)
        if nc:
            s[:nc] = self.carry_sp[:nc]
        s[nc:] = spans[:n - nc]
        al = np.where((s["has"] & 1) != 0, s["alt_len"], 0).astype(np.int64)
        ml = np.where((s["has"] & 2) != 0, s["meta_len"], 0).astype(np.int64)
        gl = np.where(inp["etype"] == EV_ALERT, inp["aux2_len"], 0).astype(np.int64)
        ln = al + ml + gl
        ln[inp["etype"] >= 16] = 0                        # control records keep their raw-batch offsets
        return ln

    def _gather_strings(self, out_recs, at, nc, spans, raw, c_sp, c_heap, L, rebase_msg):
        """The strings of partition inputs ``at`` (fresh: from ``raw``; carried: from the carry heap)
        packed back to back: (refs into the new heap, heap); an alert's message offset is rewritten
        in ``out_recs`` when ``rebase_msg``."""
        k = len(at)
        fresh = at >= nc
        s = np.zeros(k, STR_REF)
        s[fresh] = spans[at[fresh] - nc]
        s[~fresh] = c_sp[at[~fresh]]
        strip = self._strip[at]
        has = np.where(strip, s["has"] & 4, s["has"])
        al = np.where((has & 1) != 0, s["alt_len"], 0).astype(np.int64)
        ml = np.where((has & 2) != 0, s["meta_len"], 0).astype(np.int64)
        alert = out_recs["etype"] == EV_ALERT
        gl = np.where(alert & ~strip, out_recs["aux2_len"], 0).astype(np.int64)
        ctl = out_recs["etype"] >= 16
        al[ctl] = ml[ctl] = gl[ctl] = 0
        ln = al + ml + gl
        start = np.cumsum(ln) - ln
        total = int(ln.sum())
        heap = np.zeros(total, np.uint8)
        if total:
            src_heap = [np.asarray(raw, np.uint8), c_heap]
            for part, (off_f, lens) in enumerate(((s["alt_off"], al), (s["meta_off"], ml),
                                                 (out_recs["aux2_off"], gl))):
                dst0 = start + (0 if part == 0 else al if part == 1 else al + ml)
                for src_sel, src in ((fresh, src_heap[0]), (~fresh, src_heap[1])):
                    m = src_sel & (lens > 0)
                    if not m.any():
                        continue
                    ll = lens[m]
                    idx = np.repeat(off_f[m].astype(np.int64) - np.cumsum(np.concatenate([[0], ll[:-1]])), ll) + \
                        np.arange(int(ll.sum()))
                    didx = np.repeat(dst0[m] - np.cumsum(np.concatenate([[0], ll[:-1]])), ll) + np.arange(int(ll.sum()))
                    heap[didx] = src[idx]
        ns = np.zeros(k, STR_REF)
        keep = ~ctl
        ns["k"] = np.where(keep, s["k"], 0)
        ns["has"] = np.where(keep & (ln > 0), has, np.where(keep, has & 4, 0))
        ns["alt_off"] = np.where(keep & (ln > 0), start, 0)
        ns["meta_off"] = np.where(keep & (ln > 0), start + al, 0)
        ns["alt_len"] = np.where(keep & (ln > 0) & ((has & 1) != 0), s["alt_len"], 0)
        ns["meta_len"] = np.where(keep & (ln > 0) & ((has & 2) != 0), s["meta_len"], 0)
        if rebase_msg:
            am = alert & ~ctl
            out_recs["aux2_off"] = np.where(am, np.where(gl > 0, start + al + ml, 0), out_recs["aux2_off"])
            out_recs["aux2_len"] = np.where(am, gl, out_recs["aux2_len"])
        return ns, heap

    def _pack_strings(self, send, index, nc, spans, raw):
        """String slabs of a partition (``k_part_write`` in csrc/hip/swgpu.hip): per destination, each
        slab record's alternate id, metadata and alert message, from this rank's batch or the carry
        heap, copied back to back into one byte slab (the partition sized the slab's prefix to fit),
        its refs rewritten to slab offsets (the alert message offset in the record)."""
        W, S, cap = self.world, self.cfg.shuf_cap, self.cfg.str_cap
        _, c_sp, c_heap = self._part_src
        out_sp = np.zeros((W, S), STR_REF)
        buf = np.zeros(W * cap, np.uint8)
        used = np.zeros(W, np.int64)
        for o in range(W):
            at = index[o]
            k = len(at)
            if not k:
                continue
            r = send[o, :k]
            ns, heap = self._gather_strings(r, at, nc, spans, raw, c_sp, c_heap, None, rebase_msg=True)
            assert len(heap) <= cap
            buf[o * cap:o * cap + len(heap)] = heap
            used[o] = len(heap)
            out_sp[o, :k] = ns
        return out_sp, buf, used

    def _dest(self, recs: np.ndarray) -> np.ndarray:
        """Re-key destination (``part_dest`` in csrc/hip/swgpu.hip): the device's owner for a record
        whose device is registered with an active assignment (the registry is replicated on every
        rank), the decoding rank for every other record -- it holds the payload the slow path routes."""
        owner = ((recs["fp_hi"] >> np.uint64(32)) % np.uint64(self.world)).astype(np.int64)
        for i in range(len(recs)):
            if int(recs[i]["etype"]) >= 16:
                owner[i] = self.rank
                continue
            d = self.lookup_device(int(recs[i]["fp_lo"]), int(recs[i]["fp_hi"]))
            a = int(self.dev_asg[d]) if d >= 0 else -1
            if a < 0 or not self.asg_active[a]:
                owner[i] = self.rank
        return owner

    def carry_count(self) -> int:
        return len(self.carry)

    def rechecks(self, res):
        """The step's rechecks with their strings (records, refs, heap), or None (see
        ``pipeline/recheck.py``)."""
        return res.recheck

    def inject_settled(self, recs, spans, heap):
        """Re-inject records whose store-backed dedup the host settled (false positives of the
        filter) at the end of the re-key carry, with their strings; the next round processes them,
        the filter skipping them (``F_SETTLED``)."""
        from .recheck import rebase_into
        if self.world == 1:
            raise RuntimeError("settled records re-enter through the re-key carry (several ranks)")
        if (len(self.carry) + len(recs) > self.cfg.carry_cap
                or len(self.carry_heap) + len(heap) > self.cfg.carry_str_cap):
            raise RuntimeError("re-key carry full: settle after a drain round")
        r, sp = rebase_into(recs, spans, len(self.carry_heap), F_SETTLED)
        self.carry_sp = np.concatenate([self._carry_spans_full(), sp])
        self.carry = np.concatenate([self.carry, r])
        self.carry_heap = np.concatenate([self.carry_heap, np.asarray(heap, np.uint8)])

    def _carry_spans_full(self) -> np.ndarray:
        sp = self.carry_sp
        if len(sp) != len(self.carry):             # carry built without strings
            sp = np.zeros(len(self.carry), STR_REF)
        return sp

    @staticmethod
    def unpack(recv: np.ndarray, rcnt) -> np.ndarray:
        return np.concatenate([recv[q, :int(rcnt[q])] for q in range(recv.shape[0])])

    def _shuffle(self, recs: np.ndarray, raw=None):
        """Re-key of this step's records: (work batch, its string refs, their string source) -- the
        last two None when strings do not travel (custom transport, ``str_bytes`` = 0)."""
        if self.world == 1:
            return recs, None, None
        if self.exchange is not None:          # loopback / custom transport
            return self.exchange(self, recs), None, None
        import torch

        from ..parallel.sharding import exchange_slabs
        strings = bool(self.cfg.str_cap) and raw is not None and getattr(self, "_dec_spans", None) is not None
        if strings:
            send, cnt, index, nc = self.partition(recs, with_index=True, spans=self._dec_spans,
                                                  raw=np.asarray(raw, np.uint8))
        else:
            send, cnt, index, nc = self.partition(recs, with_index=True)
        extra = ()
        if strings:
            sp, sbuf, sused = self._pack_strings(send, index, nc, self._dec_spans, np.asarray(raw, np.uint8))
            rsp = np.zeros_like(sp)
            rbuf = np.zeros_like(sbuf)
            rused = np.zeros_like(sused)
            extra = ((torch.from_numpy(sused), torch.from_numpy(rused)),
                     (torch.from_numpy(sp.reshape(-1).view(np.uint8)), torch.from_numpy(rsp.reshape(-1).view(np.uint8))),
                     (torch.from_numpy(sbuf), torch.from_numpy(rbuf)))
        # the exchange carries the packed 64-byte form, like the GPU all-to-all
        send_t = torch.from_numpy(wire_pack(send.reshape(-1)).view(np.uint8))
        recv_t = torch.empty_like(send_t)
        cnt_t = torch.from_numpy(cnt)
        rcnt_t = torch.empty_like(cnt_t)
        exchange_slabs(cnt_t, rcnt_t, send_t, recv_t, self.group, extra)
        wire = recv_t.numpy().view(WIRE_REC).reshape(self.world, self.cfg.shuf_cap)
        recv = np.stack([wire_unpack(wire[q], q) for q in range(self.world)])
        rc = rcnt_t.numpy()
        work = self.unpack(recv, rc)
        if not strings:
            return work, None, None
        # refs rebased into the gathered slabs (+ source rank * str_cap), as k_unpack does
        cap = self.cfg.str_cap
        wsp = np.concatenate([rsp[q, :int(rc[q])] for q in range(self.world)])
        base = np.concatenate([np.full(int(rc[q]), q * cap, np.int64) for q in range(self.world)])
        wsp["alt_off"] = (wsp["alt_off"].astype(np.int64) + base).astype(np.uint32)
        wsp["meta_off"] = (wsp["meta_off"].astype(np.int64) + base).astype(np.uint32)
        am = work["etype"] == EV_ALERT
        work["aux2_off"] = np.where(am, (work["aux2_off"].astype(np.int64) + base).astype(np.uint32), work["aux2_off"])
        return work, wsp, rbuf

    def _lookup(self, recs):
        n = len(recs)
        status = np.zeros(n, np.uint8)
        dev = np.full(n, -1, np.int32)
        asg = np.full(n, -1, np.int32)
        for i in range(n):
            r = recs[i]
            et = int(r["etype"])
            if et == EV_DECODE_ERROR:
                status[i] = ST_DECODE_ERROR
                continue
            d = self.lookup_device(int(r["fp_lo"]), int(r["fp_hi"]))
            dev[i] = d
            if et >= 16:
                status[i] = ST_CONTROL
            elif d < 0:
                status[i] = ST_UNREGISTERED
            else:
                a = int(self.dev_asg[d])
                asg[i] = a
                status[i] = ST_OK if (a >= 0 and self.asg_active[a]) else ST_UNASSIGNED
        return status, dev, asg

    def _dedup(self, recs, status, any_rank: bool = False):
        """Generational window, the oracle of k_dedup_rotate / k_dedup_insert / k_dedup_check: ids of
        the previous generation are duplicates; otherwise the first occurrence in the current
        generation wins.  Before a batch that could push the current generation past half the
        window's slots, the generations rotate and the oldest is forgotten."""
        if len(self.dedup) + self.cfg.rec_cap > self.cfg.dedup_slots // 2:
            self.dedup_prev = self.dedup
            self.dedup = {}
            self.stats[15] += 1
        prev = self.dedup_prev
        cur = self.dedup
        for i in range(len(recs)):
            h = int(recs[i]["alt_hash"])
            # a settled recheck skips the window: its id was claimed when it came back as a recheck
            if h == 0 or status[i] != ST_OK or int(recs[i]["flags"]) & F_SETTLED:
                continue
            if h in prev or h in cur:
                status[i] = ST_DUPLICATE
            else:
                cur[h] = self.seq_base + i
                # maybe stored before: the host checks.  The filter sees every record this rank
                # owns when their strings came along (``any_rank``: the host settles a recheck by its
                # alternate id), else only records decoded here (the host path re-reads their
                # payload); a record the host already settled skips it
                if (self.ff is not None and not (int(recs[i]["flags"]) & F_SETTLED)
                        and (any_rank or int(recs[i]["src_rank"]) == self.rank) and self.ff.has(h)):
                    status[i] = ST_RECHECK

    def reset_dedup(self):
        """Forget the alternate-id window (both generations); the store-backed filter stays."""
        self.dedup, self.dedup_prev = {}, {}
        self.dedup_valid_from = self.cursor           # the window holds no id of the rows before

    # store-backed filter primitives (EngineBase.filter_seed / filter_state)
    def _ff_meta_get(self) -> np.ndarray:
        return self.ff.meta.copy()

    def _ff_meta_set(self, m):
        self.ff.meta[:] = m

    def _ff_add(self, hashes, g: int):
        for h in np.asarray(hashes, np.uint64).tolist():
            if h:
                self.ff.add(int(h), g)

    def _ff_clear(self, g: int):
        self.ff.clear(g)

    def _intern_id(self, h: int) -> int:
        if h not in self.intern:
            self.intern[h] = len(self.intern)
        return self.intern[h]

    def _persist(self, recs, dev, asg, now_ms, out_rows):
        for j in range(len(recs)):
            r = recs[j]
            seq = self.cursor + j
            row = seq % self.cfg.store_cap
            a = int(asg[j])
            s = self.store
            s["etype"][row] = r["etype"]
            s["level"][row] = r["level"]
            s["date"][row] = r["event_date"]
            s["recv"][row] = now_ms
            s["dev"][row] = dev[j]
            s["asg"][row] = a
            s["cust"][row] = self.asg_customer[a]
            s["area"][row] = self.asg_area[a]
            s["asset"][row] = self.asg_asset[a]
            s["name"][row] = r["name_hash"]
            s["v0"][row] = r["v0"]
            s["v1"][row] = r["v1"]
            s["v2"][row] = r["v2"]
            s["alt"][row] = r["alt_hash"]
            s["aux"][row] = (int(r["src_rank"]) << 48) | (int(r["aux_len"]) << 32) | int(r["aux_off"])
            s["batch"][row] = self.batch_seq
            h = int(r["name_hash"])
            nid = self.intern.get(h, -1) if h else -1
            out_rows.append((int(r["event_date"]), float(r["v0"]), float(r["v1"]), a,
                             nid if 0 <= nid < 0xFFFF else 0xFFFF, int(r["etype"]), int(r["level"])))

    def _state(self, recs, asg, now_ms):
        base = self.cursor
        for j in range(len(recs)):
            r = recs[j]
            et = int(r["etype"])
            if et not in (EV_MEASUREMENT, EV_LOCATION, EV_ALERT):
                continue
            a = int(asg[j])
            self.st_last[a] = max(int(self.st_last[a]), now_ms)
            self.st_missing[a] = 0
            d = int(r["event_date"])
            eid1 = (base + j) * self.world + self.rank + 1
            if et == EV_LOCATION:
                if d > int(self.st_loc_date[a]):
                    self.st_loc_date[a] = d
                    self.st_loc_eid[a] = eid1
                elif d == int(self.st_loc_date[a]):
                    self.st_loc_eid[a] = max(int(self.st_loc_eid[a]), eid1)
            elif int(r["name_hash"]):
                key = (a, self.intern[int(r["name_hash"])], 1 if et == EV_ALERT else 0)
                cur = self.ms.get(key)
                if cur is None or d > cur[0]:
                    self.ms[key] = [d, eid1]
                elif d == cur[0]:
                    cur[1] = max(cur[1], eid1)

    # ------------------------------------------------------------------ step
    def step(self, raw: np.ndarray, offs: np.ndarray, now_ms: int, presence: bool | None = None) -> StepResult:
        recs, new = self.decode_phase(raw, offs, now_ms)
        # strings: this rank's batch on one rank; the exchanged string slabs on several
        work, spans, src = self._shuffle(recs, raw)
        if self.world == 1:
            spans, src = self._dec_spans, raw
        res = self.process_phase(work, len(offs) - 1, now_ms, new, presence, spans=spans)
        if spans is not None:
            res.raw = src
            if self.world > 1:
                # the owner settles them by alternate id: their strings, before the block encoder
                # lets go of the string source
                from .recheck import host_rechecks
                res.recheck = host_rechecks(res)
        return res

    def decode_phase(self, raw, offs, now_ms):
        recs, self._dec_spans = cpu_decode(raw, offs, now_ms, self.rank, cap=self.cfg.rec_cap, spans=True)
        # new-name capture on the source rank
        refs = []
        for r in recs:
            h = int(r["name_hash"])
            if h and r["etype"] < 16 and h not in self._seen:
                self._seen.add(h)
                refs.append((h, int(r["aux_off"]), int(r["aux_len"]), int(r["src_rank"]), int(r["etype"])))
        from ..models.columnar import NAME_REF
        new = self.learn_names(np.array(refs, NAME_REF), raw) if refs else {}
        return recs, new

    def process_phase(self, work, n_msgs, now_ms, new, presence=None, spans=None) -> StepResult:
        first_seq = self.cursor
        status, dev, asg = self._lookup(work)
        self._dedup(work, status, any_rank=self.world > 1 and spans is not None)
        ok = np.nonzero(status == ST_OK)[0]
        rej = np.nonzero(status != ST_OK)[0]
        for i in ok:
            h = int(work[i]["name_hash"])
            if h:
                self._intern_id(h)
        if self.cfg.cluster and len(ok) > 1:
            # persist order: stable by assignment (the durable block's clustering, swindex.h)
            ok = ok[np.argsort(asg[ok], kind="stable")]
        out_rows: list = []
        self._persist(work[ok], dev[ok], asg[ok], now_ms, out_rows)
        if self.ff is not None:                          # persisted ids join the filter's live generation
            self.ff.add_persisted(work[ok]["alt_hash"])
        self._state(work[ok], asg[ok], now_ms)
        self.cursor += len(ok)
        # rules on persisted locations
        gen, gen_dev, gen_asg = [], [], []
        if self.tests:
            vtx, zoff, _, tests, hashes = self.zone_arrays()
            polys = [vtx.reshape(-1, 2)[zoff[z]:zoff[z + 1]] for z in range(len(zoff) - 1)]
            for o in out_rows:
                if o[5] != EV_LOCATION:
                    continue
                for t, zt in enumerate(tests):
                    inside = pip(polys[int(zt["zone"])], o[1], o[2])
                    if (int(zt["condition"]) == 0) == inside:
                        if len(gen) < self.cfg.gen_cap:
                            gen.append((0, 0, now_ms, int(hashes[t]), 0.0, 0.0, 0.0, 0, t, 0, 0, 0, EV_ALERT, 0,
                                        self.rank, int(zt["level"])))
                            gen_dev.append(int(self.asg_device[o[3]]))
                            gen_asg.append(o[3])
        n_rule = len(gen)
        do_presence = self.presence_due(now_ms) if presence is None else presence
        if do_presence and self.cfg.presence_missing_ms > 0:
            limit = now_ms - self.cfg.presence_missing_ms
            miss = np.nonzero((self.asg_active[:self.n_assignments] > 0) & (self.st_last[:self.n_assignments] > 0) &
                              (self.st_last[:self.n_assignments] < np.uint64(max(limit, 0))) &
                              (self.st_missing[:self.n_assignments] == 0))[0]
            for a in miss:
                self.st_missing[a] = now_ms
                if len(gen) < self.cfg.gen_cap:
                    gen.append((0, 0, now_ms, self.presence_hash, 0.0, 0.0, 0.0, 0, 0, 0, 0, 0, EV_STATE_CHANGE, 0,
                                self.rank, 0))
                    gen_dev.append(int(self.asg_device[a]))
                    gen_asg.append(int(a))
        g = np.zeros(0, EVENT_REC)
        if gen:
            g = np.array(gen, EVENT_REC)
            for r in g:
                if int(r["name_hash"]):
                    self._intern_id(int(r["name_hash"]))
            gd = np.asarray(gen_dev, np.int32)
            ga = np.asarray(gen_asg, np.int32)
            self._persist(g, gd, ga, now_ms, out_rows)
            self._state(g, ga, now_ms)
            self.cursor += len(g)
        if self.ff is not None:
            self.ff.end_step(self.cursor)
        # bookkeeping
        self.seq_base += len(work)
        st = self.stats
        st[0] += n_msgs
        st[1] += len(work)
        st[2] += len(out_rows)
        for code, slot in ((ST_UNREGISTERED, 3), (ST_UNASSIGNED, 4), (ST_DUPLICATE, 5), (ST_DECODE_ERROR, 6),
                           (ST_CONTROL, 7), (ST_RECHECK, 16)):
            st[slot] += int((status == code).sum())
        st[8] += n_rule
        st[9] += len(gen) - n_rule
        st[11] += len(new)
        self.batch_seq += 1
        prec = np.concatenate([work[ok], g])
        pspans = np.concatenate([spans[ok], np.zeros(len(g), STR_REF)]) if spans is not None else None
        return StepResult(n_msgs=n_msgs, n_events=len(work), n_persisted=len(out_rows),
                          out=np.array(out_rows, OUT_REC), rejects=work[rej], reject_status=status[rej],
                          new_names=new, first_seq=first_seq, world=self.world, rank=self.rank, prec=prec,
                          pspans=pspans, rspans=spans[rej] if spans is not None and self.world > 1 else None)

    # ------------------------------------------------------------------ checkpoint / resume
    kind = "cpu"

    def checkpoint_state(self, include_store: bool = False) -> dict:
        u64 = lambda xs: np.array(list(xs), np.uint64)  # noqa: E731
        ms_keys = list(self.ms.keys())
        st = {
            "scalars": np.array([self.cursor, self.seq_base], np.int64),
            "stats": self.stats.copy(),
            "dedup_key": u64(self.dedup.keys()), "dedup_seq": np.array(list(self.dedup.values()), np.int64),
            "dedup_prev_key": u64(self.dedup_prev.keys()),
            "dedup_prev_seq": np.array(list(self.dedup_prev.values()), np.int64),
            **(dict(zip(("dd_ff_idx", "dd_ff_rows"), self.ff.export()), dd_ff_meta=self.ff.meta.copy())
               if self.ff is not None else {}),
            "intern_key": u64(self.intern.keys()), "intern_id": np.array(list(self.intern.values()), np.int64),
            "seen": u64(self._seen),
            "st_last": self.st_last, "st_missing": self.st_missing, "st_loc_date": self.st_loc_date,
            "st_loc_eid": self.st_loc_eid,
            "ms_key": np.array(ms_keys, np.int64).reshape(-1, 3),
            "ms_val": np.array([self.ms[k] for k in ms_keys], np.int64).reshape(-1, 2),
            "carry": self.carry.view(np.uint8).reshape(-1).copy(),
            "carry_spans": self._carry_spans_full().view(np.uint8).reshape(-1).copy(),
            "carry_str": self.carry_heap.copy(),
        }
        if include_store:
            st.update({f"store.{k}": v for k, v in self.store.items()})
        return st

    def restore_state(self, a: dict, include_store: bool):
        self.cursor, self.seq_base = (int(x) for x in a["scalars"])
        self.stats[:] = 0
        self.stats[:len(a["stats"])] = a["stats"]
        if self.ff is not None and "dd_ff_idx" in a:
            self.ff.load(a["dd_ff_idx"], a["dd_ff_rows"])
            self.ff.meta[:] = a["dd_ff_meta"]
        self.dedup = dict(zip((int(x) for x in a["dedup_key"]), (int(x) for x in a["dedup_seq"])))
        self.dedup_prev = dict(zip((int(x) for x in a.get("dedup_prev_key", [])),
                                   (int(x) for x in a.get("dedup_prev_seq", []))))
        self.intern = dict(zip((int(x) for x in a["intern_key"]), (int(x) for x in a["intern_id"])))
        self._seen = {int(x) for x in a["seen"]}
        for k in ("st_last", "st_missing", "st_loc_date", "st_loc_eid"):
            getattr(self, k)[:] = a[k]
        self.ms = {tuple(int(x) for x in k): [int(v[0]), int(v[1])] for k, v in zip(a["ms_key"], a["ms_val"])}
        self.carry = a["carry"].view(EVENT_REC).copy()
        # the carry's strings (an older checkpoint has none: its records go without them)
        self.carry_sp = (a["carry_spans"].view(STR_REF).copy() if "carry_spans" in a
                         else np.zeros(len(self.carry), STR_REF))
        self.carry_heap = a.get("carry_str", np.zeros(0, np.uint8)).copy()
        if include_store:
            for k in self.store:
                self.store[k][:] = a[f"store.{k}"]

    # ------------------------------------------------------------------ queries
    def stats_dict(self) -> dict:  # type: ignore[override]
        return {n: int(self.stats[i]) for i, n in enumerate(STAT_NAMES)}

    def device_state(self, asg: int) -> dict:
        mx = {}
        al = {}
        inv = {v: k for k, v in self.intern.items()}
        for (a, nid, kind), (d, e1) in self.ms.items():
            if a != asg:
                continue
            name = self.names.get(inv[nid], str(inv[nid]))
            (al if kind else mx)[name] = (e1 - 1, d)
        return {
            "assignment": asg,
            "last_interaction": int(self.st_last[asg]),
            "presence_missing": int(self.st_missing[asg]),
            "last_location": (int(self.st_loc_eid[asg]) - 1, int(self.st_loc_date[asg])) if self.st_loc_eid[asg] else None,
            "measurements": mx,
            "alerts": al,
        }

    def query_store(self, event_type, asg_idx, start=None, end=None, page_number=1, page_size=100):
        n = min(self.cursor, self.cfg.store_cap)
        s = self.store
        m = s["etype"][:n] == event_type
        m &= np.isin(s["asg"][:n], np.asarray(list(asg_idx), np.int32))
        d = s["date"][:n]
        if start is not None:
            m &= d >= start
        if end is not None:
            m &= d <= end
        rows = np.nonzero(m)[0]
        seq = self._row_seq(rows.astype(np.int64), self.cursor)
        order = np.lexsort((-seq, -d[rows]))
        lo, hi = self._window(page_number, page_size, len(rows))
        page = rows[order[lo:hi]]
        cols = {k: v[page] for k, v in s.items()}
        return len(rows), cols, seq[order[lo:hi]] * self.world + self.rank

    def intern_table(self) -> dict:
        """name hash -> dense name id (same form as the GPU and native engines)."""
        return dict(self.intern)

    def store_rows(self):
        n = min(self.cursor, self.cfg.store_cap)
        if self.cursor <= self.cfg.store_cap:
            idx = np.arange(n)
        else:
            start = self.cursor % self.cfg.store_cap
            idx = (np.arange(n) + start) % self.cfg.store_cap
        return {k: v[idx] for k, v in self.store.items()}, (np.arange(self.cursor - n, self.cursor) * self.world + self.rank)
