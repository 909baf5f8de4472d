"""Native CPU engine shard: the fused inbound pipeline on host cores (``csrc/native/swcpuengine.cpp``).

Same interface and the same results, bit for bit, as the Python oracle :class:`CpuInboundEngine`
(``tests/test_native_engine.py`` checks store, outbound rows, device state, dedup and stats after
multi-step fleets).  The oracle stays the readable specification and the parity reference; this
engine is what a tenant without an MI355X runs (``device: "cpu"`` / ``"auto"``) and what
``bench.py --engine cpu`` measures, so the GPU numbers are compared against a competent
multi-threaded CPU implementation of the same design rather than against a Python loop.

Reference counterparts: the per-event services the engine fuses (see ``engine_base``).
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

from .._native import native
from ..models.columnar import EVENT_REC, N_STATS, NAME_REF, OUT_REC, REG_SLOT, STAT_NAMES, STR_REF
from .config import EngineConfig
from .cpu_engine import STORE_COLS, CpuInboundEngine
from .engine_base import EngineBase, StepResult
from .fleet import cpu_decode

_P = ctypes.c_void_p


# SwCeState: per-assignment device state, one 32-byte row (the oracle keeps four arrays; here they
# are strided views of this table so both engines expose the same ``st_*`` attributes)
ASG_STATE = np.dtype([("last", "<u8"), ("missing", "<u8"), ("loc_date", "<u8"), ("loc_eid", "<i8")])


class _Tables(ctypes.Structure):
    """``SwCeTables`` (swcpuengine.cpp)."""
    _fields_ = [("reg", _P), ("reg_mask", ctypes.c_int64), ("ctx", _P), ("asg_active", _P),
                ("n_assignments", ctypes.c_int64), ("st", _P)] + \
        [(f"s_{k}", _P) for k in STORE_COLS] + [("store_cap", ctypes.c_int64)] + \
        [(n, _P) for n in ("zone_vtx", "zone_off", "zone_bbox", "tests", "test_hash")] + \
        [("n_tests", ctypes.c_int32), ("rank", ctypes.c_int32), ("world", ctypes.c_int32),
         ("batch_seq", ctypes.c_int32), ("gen_cap", ctypes.c_int64), ("presence_hash", ctypes.c_uint64),
         ("presence_missing_ms", ctypes.c_int64), ("stats", _P), ("cluster", ctypes.c_int32),
         ("pad0", ctypes.c_int32)]


class _Step(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int64) for n in ("cursor", "seq_base", "n_ok", "n_gen", "n_rule", "n_rej")]


def default_threads() -> int:
    env = os.environ.get("SW_CPU_ENGINE_THREADS")
    if env:
        return max(1, min(64, int(env)))
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(64, n))


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


class NativeCpuEngine(CpuInboundEngine):
    """Multi-threaded C++ engine shard; host tables stay numpy (shared with the control plane)."""

    kind = "cpu"

    def __init__(self, cfg: EngineConfig, group=None, threads: int | None = None):
        EngineBase.__init__(self, cfg)
        self.group = group
        self.exchange = None
        self.carry = np.zeros(0, EVENT_REC)
        self.carry_sp = np.zeros(0, STR_REF)        # the carry's strings (CpuInboundEngine.partition)
        self.carry_heap = np.zeros(0, np.uint8)
        self.str_drops = [0, 0]
        self.store = {k: np.zeros(cfg.store_cap, t) for k, t in STORE_COLS.items()}
        self.cursor = 0
        self.seq_base = 0
        self._st = np.zeros(cfg.max_assignments, ASG_STATE)
        self.st_last, self.st_missing = self._st["last"], self._st["missing"]
        self.st_loc_date, self.st_loc_eid = self._st["loc_date"], self._st["loc_eid"]
        # packed mirrors the native stages read (kept current by the EngineBase dirty hooks)
        self.reg_packed = np.zeros(cfg.reg_slots, REG_SLOT)
        self.asg_ctx = np.full((cfg.max_assignments, 4), -1, np.int32)   # device, customer, area, asset
        self.stats = np.zeros(N_STATS, np.uint64)
        self.threads = threads or default_threads()
        self._lib = native()
        self._h = self._lib.swce_create(self.threads)
        self._lib.swce_reserve(self._h, cfg.state_slots, cfg.dedup_slots)
        self._lib.swce_dedup_window(self._h, cfg.dedup_slots, cfg.rec_cap)
        if self._lib.swce_ff_init(self._h, cfg.ff_buckets, cfg.dedup_filter_gens if cfg.ff_buckets else 0,
                                  cfg.dedup_filter_ids) != 0:
            raise MemoryError("store-backed dedup filter: bad sizing or out of memory")
        for v in self.store.values():      # touch the ring now (the GPU's HBM store is resident too)
            v.fill(0)
        self._out_pool: dict = {}       # recycled outbound buffers per dtype (see _out_buffer)
        self._status = np.zeros(cfg.rec_cap, np.uint8)
        self._zones = None
        self._zones_changed()
        self._dec, self._dec_k = [None, None], 0
        self._dsp = [None, None]

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._lib.swce_destroy(h)
            self._h = None

    def reset_dedup(self):
        """Forget the alternate-id window (both generations); the store-backed filter stays."""
        self.dedup_valid_from = self.cursor           # the window holds no id of the rows before
        z64, zi = np.zeros(1, np.uint64), np.zeros(1, np.int64)
        self._lib.swce_dedup_import(self._h, _ptr(z64), _ptr(zi), 0)
        self._lib.swce_dedup_prev_import(self._h, _ptr(z64), _ptr(zi), 0)

    # store-backed filter primitives (EngineBase.filter_seed / filter_state)
    def _ff_meta_get(self) -> np.ndarray:
        m = np.zeros(24, np.int64)
        self._lib.swce_ff_meta(self._h, _ptr(m), None)
        return m

    def _ff_meta_set(self, m):
        m = np.ascontiguousarray(np.asarray(m, np.int64))
        self._lib.swce_ff_meta(self._h, None, _ptr(m))

    def _ff_add(self, hashes, g: int):
        h = np.ascontiguousarray(np.asarray(hashes, np.uint64))
        if len(h):
            self._lib.swce_ff_add(self._h, int(g), _ptr(h), len(h))

    def _ff_clear(self, g: int):
        self._lib.swce_ff_clear(self._h, int(g))

    # ------------------------------------------------------------------ packed mirrors
    def _dirty_registry(self, slots):
        slots = np.asarray(slots, np.int64)
        slots = slots[slots >= 0]
        if len(slots):
            self.reg_packed[slots] = self.packed_registry(slots)

    def _dirty_devices(self, idx):
        self._dirty_registry(self.dev_slot[np.asarray(idx, np.int64)])

    def _dirty_assignments(self, idx):
        idx = np.asarray(idx, np.int64)
        self.asg_ctx[idx, 0] = self.asg_device[idx]
        self.asg_ctx[idx, 1] = self.asg_customer[idx]
        self.asg_ctx[idx, 2] = self.asg_area[idx]
        self.asg_ctx[idx, 3] = self.asg_asset[idx]
        dev = self.asg_device[idx]
        self._dirty_devices(dev[dev >= 0])

    def _zones_changed(self):
        self._zones = self.zone_arrays() if self.tests else None

    # ------------------------------------------------------------------ phases
    def decode_phase(self, raw, offs, now_ms):
        # two decode buffers, alternating: a batch's records stay valid while the next one decodes
        self._dec_k ^= 1
        if self._dec[self._dec_k] is None:
            self._dec[self._dec_k] = np.empty(self.cfg.rec_cap, EVENT_REC)
        if self._dsp[self._dec_k] is None:
            self._dsp[self._dec_k] = np.empty(self.cfg.rec_cap, STR_REF)
        recs, self._dec_spans = cpu_decode(raw, offs, now_ms, self.rank, threads=self.threads,
                                           out=self._dec[self._dec_k], spans=self._dsp[self._dec_k])
        refs = np.zeros(self.cfg.names_cap, NAME_REF)
        n = self._lib.swce_capture_names(self._h, _ptr(recs), len(recs), _ptr(refs), len(refs)) if len(recs) else 0
        new = self.learn_names(refs[:n], raw) if n else {}
        return recs, new

    def _tables(self) -> _Tables:
        t = _Tables()
        t.reg, t.reg_mask = _ptr(self.reg_packed), self.cfg.reg_slots - 1
        t.ctx, t.asg_active, t.st = _ptr(self.asg_ctx), _ptr(self.asg_active), _ptr(self._st)
        t.n_assignments = self.n_assignments
        for k, v in self.store.items():
            setattr(t, f"s_{k}", _ptr(v))
        t.store_cap = self.cfg.store_cap
        if self._zones is not None:
            vtx, zoff, bbox, tests, hashes = self._zones
            self._zone_keep = (vtx, zoff, bbox, tests, hashes)
            t.zone_vtx, t.zone_off, t.zone_bbox = _ptr(vtx), _ptr(zoff), _ptr(bbox)
            t.tests, t.test_hash, t.n_tests = _ptr(tests), _ptr(hashes), len(tests)
        t.rank, t.world, t.batch_seq = self.rank, self.world, self.batch_seq
        t.gen_cap = self.cfg.gen_cap
        t.presence_hash = self.presence_hash
        t.presence_missing_ms = self.cfg.presence_missing_ms
        t.cluster = 1 if self.cfg.cluster else 0
        t.stats = _ptr(self.stats)
        return t

    def process_phase(self, work, n_msgs, now_ms, new, presence=None, spans=None) -> StepResult:
        work = np.ascontiguousarray(work)
        n = len(work)
        if n > len(self._status):
            self._status = np.zeros(n, np.uint8)
        out = self._out_buffer(n + self.cfg.gen_cap)
        # persisted records + string refs, row-aligned with out (the block encoder's input); fresh
        # per step: a StepResult keeps them until its block is encoded
        prec = self._out_buffer(n + self.cfg.gen_cap, EVENT_REC)
        pspans = self._out_buffer(n + self.cfg.gen_cap, STR_REF) if spans is not None else None
        do_presence = self.presence_due(now_ms) if presence is None else presence
        first_seq = self.cursor
        st = _Step(cursor=self.cursor, seq_base=self.seq_base)
        with self._lock:
            t = self._tables()
            rc = self._lib.swce_process(self._h, ctypes.byref(t), ctypes.byref(st), _ptr(work) if n else 0, n, now_ms,
                                        1 if do_presence else 0, _ptr(self._status), _ptr(out),
                                        _ptr(spans) if spans is not None and n else 0, _ptr(prec),
                                        _ptr(pspans) if pspans is not None else 0)
        if rc != 0:
            raise RuntimeError(f"swce_process failed ({rc})")
        self.cursor, self.seq_base = st.cursor, st.seq_base
        self.stats[0] += n_msgs
        self.stats[11] += len(new)
        self.batch_seq += 1
        status = self._status[:n]
        rej = np.nonzero(status != 0)[0]
        n_out = st.n_ok + st.n_gen
        return StepResult(n_msgs=n_msgs, n_events=n, n_persisted=n_out, out=out[:n_out],
                          rejects=work[rej], reject_status=status[rej].copy(), new_names=new, first_seq=first_seq,
                          world=self.world, rank=self.rank, prec=prec[:n_out],
                          pspans=pspans[:n_out] if pspans is not None else None,
                          rspans=spans[rej] if spans is not None and self.world > 1 else None)

    def _out_buffer(self, n: int, dtype=OUT_REC) -> np.ndarray:
        """An outbound buffer (rows, or the rows' records / string refs) no earlier StepResult still
        references (checked by refcount: a live ``result.out`` view pins its base), so results need
        no copy and no fresh pages per step."""
        pool = self._out_pool.setdefault(np.dtype(dtype).str + str(np.dtype(dtype).itemsize), [])
        for b in pool:
            if len(b) >= n and sys.getrefcount(b) <= 3:    # the pool list, the loop variable, the call
                return b
        b = np.empty(max(n, self.cfg.rec_cap + self.cfg.gen_cap), dtype)
        if len(pool) < 4:
            pool.append(b)
        return b

    # ------------------------------------------------------------------ native tables
    def intern_table(self) -> dict:
        n = self._lib.swce_intern_size(self._h)
        keys, ids = np.zeros(n, np.uint64), np.zeros(n, np.int32)
        if n:
            self._lib.swce_intern_export(self._h, _ptr(keys), _ptr(ids))
        return {int(k): int(i) for k, i in zip(keys, ids)}

    def _ms_rows(self) -> np.ndarray:
        n = self._lib.swce_ms_size(self._h)
        rows = np.zeros((n, 5), np.int64)
        if n:
            self._lib.swce_ms_export(self._h, _ptr(rows))
        return rows

    def checkpoint_state(self, include_store: bool = False) -> dict:
        lib, h = self._lib, self._h
        nd = lib.swce_dedup_size(h)
        dk, ds = np.zeros(nd, np.uint64), np.zeros(nd, np.int64)
        if nd:
            lib.swce_dedup_export(h, _ptr(dk), _ptr(ds))
        npv = lib.swce_dedup_prev_size(h)
        pk, ps = np.zeros(npv, np.uint64), np.zeros(npv, np.int64)
        if npv:
            lib.swce_dedup_prev_export(h, _ptr(pk), _ptr(ps))
        intern = self.intern_table()
        ns = lib.swce_seen_size(h)
        seen = np.zeros(ns, np.uint64)
        if ns:
            lib.swce_seen_export(h, _ptr(seen))
        ms = self._ms_rows()
        st = {
            "scalars": np.array([self.cursor, self.seq_base], np.int64),
            "stats": self.stats.copy(),
            "dedup_key": dk, "dedup_seq": ds, "dedup_prev_key": pk, "dedup_prev_seq": ps,
            "intern_key": np.array(list(intern.keys()), np.uint64),
            "intern_id": np.array(list(intern.values()), np.int64),
            "seen": seen,
            "st_last": self.st_last, "st_missing": self.st_missing, "st_loc_date": self.st_loc_date,
            "st_loc_eid": self.st_loc_eid,
            "ms_key": ms[:, :3].copy(), "ms_val": ms[:, 3:].copy(),
            "carry": self.carry.view(np.uint8).reshape(-1).copy(),
        }
        if self.filter_on:
            n = int(lib.swce_ff_export(h, None, None, 0))
            idx, rows = np.zeros(max(n, 1), np.int64), np.zeros((max(n, 1), 16), np.uint32)
            lib.swce_ff_export(h, _ptr(idx), _ptr(rows), n)
            st["dd_ff_idx"], st["dd_ff_rows"] = idx[:n], rows[:n]
            st["dd_ff_meta"] = self._ff_meta_get()
        if include_store:
            st.update({f"store.{k}": v for k, v in self.store.items()})
        return st

    def restore_state(self, a: dict, include_store: bool):
        lib, h = self._lib, self._h
        if "dd_ff_idx" in a and self.filter_on:
            idx = np.ascontiguousarray(a["dd_ff_idx"], np.int64)
            rows = np.ascontiguousarray(a["dd_ff_rows"], np.uint32).reshape(-1, 16)
            if lib.swce_ff_import(h, _ptr(idx), _ptr(rows), len(idx)) != 0:
                raise ValueError("checkpoint's dedup filter does not fit this engine's filter")
            self._ff_meta_set(a["dd_ff_meta"])
        self.cursor, self.seq_base = (int(x) for x in a["scalars"])
        self.stats[:] = 0
        self.stats[:len(a["stats"])] = a["stats"]
        dk = np.ascontiguousarray(a["dedup_key"], np.uint64)
        ds = np.ascontiguousarray(a["dedup_seq"], np.int64)
        lib.swce_dedup_import(h, _ptr(dk), _ptr(ds), len(dk))
        pk = np.ascontiguousarray(a.get("dedup_prev_key", np.zeros(0, np.uint64)), np.uint64)
        ps = np.ascontiguousarray(a.get("dedup_prev_seq", np.zeros(0, np.int64)), np.int64)
        lib.swce_dedup_prev_import(h, _ptr(pk), _ptr(ps), len(pk))
        ik = np.ascontiguousarray(a["intern_key"], np.uint64)
        ii = np.ascontiguousarray(a["intern_id"], np.int32)
        lib.swce_intern_import(h, _ptr(ik), _ptr(ii), len(ik))
        sk = np.ascontiguousarray(a["seen"], np.uint64)
        lib.swce_seen_import(h, _ptr(sk), len(sk))
        for k in ("st_last", "st_missing", "st_loc_date", "st_loc_eid"):
            getattr(self, k)[:] = a[k]
        rows = np.ascontiguousarray(np.concatenate([np.asarray(a["ms_key"], np.int64).reshape(-1, 3),
                                                    np.asarray(a["ms_val"], np.int64).reshape(-1, 2)], axis=1))
        lib.swce_ms_import(h, _ptr(rows), len(rows))
        self.carry = a["carry"].view(EVENT_REC).copy()
        if include_store:
            for k in self.store:
                self.store[k][:] = a[f"store.{k}"]

    # ------------------------------------------------------------------ queries
    def stats_dict(self) -> dict:  # type: ignore[override]
        return {n: int(self.stats[i]) for i, n in enumerate(STAT_NAMES)}

    def device_state(self, asg: int) -> dict:
        rows = np.zeros((4096, 4), np.int64)
        n = self._lib.swce_ms_of(self._h, int(asg), _ptr(rows), len(rows))
        inv = {v: k for k, v in self.intern_table().items()}
        mx, al = {}, {}
        for nid, kind, d, e1 in rows[:n]:
            hsh = inv[int(nid)]
            name = self.names.get(hsh, str(hsh))
            (al if kind else mx)[name] = (int(e1) - 1, int(d))
        return {
            "assignment": asg,
            "last_interaction": int(self.st_last[asg]),
            "presence_missing": int(self.st_missing[asg]),
            "last_location": (int(self.st_loc_eid[asg]) - 1, int(self.st_loc_date[asg])) if self.st_loc_eid[asg] else None,
            "measurements": mx,
            "alerts": al,
        }
