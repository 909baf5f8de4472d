"""Host-side state shared by the GPU and CPU inbound-pipeline engines.

An *engine shard* owns one tenant's hot data on one rank: the device registry
(token fingerprint -> device index), the active assignment and its context
(customer / area / asset), the HBM event store, device state, the dedup window,
the zone-test rules and the presence settings.  The control plane (device
management service) pushes registry / assignment / zone changes here; the data
plane (``step``) consumes raw payload batches.

Reference counterparts: the per-tenant engines of service-inbound-processing,
service-event-management, service-device-state and service-rule-processing
(``*TenantEngine.java``), collapsed into one fused micro-batch pipeline.
"""
from __future__ import annotations

import threading
from dataclasses import dataclass, field

import numpy as np

from .._native import native
from ..models.columnar import OUT_REC, STAT_NAMES, REG_SLOT
from .config import EngineConfig
from .fleet import hash64


def _p(a: np.ndarray) -> int:
    return a.ctypes.data


@dataclass
class Zone:
    """A polygon zone; vertices are (latitude, longitude) pairs (reference IZone bounds)."""
    token: str
    vertices: list


@dataclass
class ZoneTest:
    """Zone-test rule (reference: service-rule-processing/.../geospatial/ZoneTest.java)."""
    zone_token: str
    condition: str = "inside"       # "inside" | "outside" (ZoneContainment)
    alert_type: str = "zone.alert"
    alert_level: int = 1            # Info=0, Warning=1, Error=2, Critical=3
    alert_message: str = ""


@dataclass
class StepResult:
    """What one micro-batch produced (host copies; filled by ``finalize``)."""
    n_msgs: int = 0
    n_events: int = 0
    n_persisted: int = 0
    out: np.ndarray | None = None          # OUT_REC rows (persisted, enriched)
    rejects: np.ndarray | None = None      # EVENT_REC rows not persisted
    reject_status: np.ndarray | None = None
    new_names: dict = field(default_factory=dict)
    first_seq: int = 0                     # store sequence of out[0]; ids are implicit
    world: int = 1
    rank: int = 0
    # (buffer, offset) when ``out`` sits at ``offset`` of a pooled pinned buffer with free bytes in
    # front of it: a columnar batch can be framed around the rows in place (``frame_columnar``)
    frame_base: tuple | None = None
    # the step's sealed durable block (``persistence/segments.py``) when the engine encodes blocks
    # (``encode_blocks``); ``block_frame`` = (buffer, offset) as for ``frame_base``
    block: np.ndarray | None = None
    block_frame: tuple | None = None
    # host engines: what the durable-block encoder needs beside ``out`` -- the persisted records and
    # their string refs (row-aligned with ``out``) and the raw batch the strings live in (dropped
    # once the block is encoded: it may view a topic record)
    prec: np.ndarray | None = None
    pspans: np.ndarray | None = None
    raw: np.ndarray | None = None
    # several ranks, strings exchanged: string refs of ``rejects`` (into ``raw``: host engines) or
    # the step's rechecks with their strings (records, refs, heap: MI355X engine), which the owner
    # settles by alternate id (``pipeline/recheck.py``)
    rspans: np.ndarray | None = None
    recheck: tuple | None = None

    def event_ids(self) -> np.ndarray:
        n = 0 if self.out is None else len(self.out)
        return (self.first_seq + np.arange(n, dtype=np.int64)) * self.world + self.rank


class EngineBase:
    """Registry / assignment / zone mirrors + names dictionary (host side)."""

    PRESENCE = "presence"

    def __init__(self, cfg: EngineConfig):
        self.cfg = cfg
        self.rank, self.world = cfg.rank, cfg.world
        self._lock = threading.RLock()
        # registry mirror (exact 128-bit keys)
        self.reg_lo = np.zeros(cfg.reg_slots, np.uint64)
        self.reg_hi = np.zeros(cfg.reg_slots, np.uint64)
        self.reg_val = np.full(cfg.reg_slots, -1, np.int32)
        self.n_devices = 0
        self.dev_slot = np.full(cfg.max_devices, -1, np.int64)   # registry slot of each device
        self.dev_asg = np.full(cfg.max_devices, -1, np.int32)
        self.dev_type = np.full(cfg.max_devices, -1, np.int32)
        self.asg_device = np.full(cfg.max_assignments, -1, np.int32)
        self.asg_customer = np.full(cfg.max_assignments, -1, np.int32)
        self.asg_area = np.full(cfg.max_assignments, -1, np.int32)
        self.asg_asset = np.full(cfg.max_assignments, -1, np.int32)
        self.asg_active = np.zeros(cfg.max_assignments, np.uint8)
        self.n_assignments = 0
        # names: global hash -> string dictionary
        self.names: dict[int, str] = {}
        self.presence_hash = hash64(self.PRESENCE)
        self.names[self.presence_hash] = self.PRESENCE
        # zones
        self.zones: list[Zone] = []
        self.tests: list[ZoneTest] = []
        self.batch_seq = 0
        self.presence_enabled = True
        self._last_presence_check = None

    # ------------------------------------------------------------------ registry
    def _dirty_registry(self, slots: np.ndarray):
        """Hook: GPU engine pushes changed slots to HBM."""

    def _dirty_assignments(self, idx: np.ndarray):
        """Hook: GPU engine pushes changed assignment rows."""

    def _dirty_devices(self, idx: np.ndarray):
        """Hook: GPU engine pushes changed device rows."""

    def register_devices(self, fp_lo, fp_hi, dev_idx=None, dev_type=None) -> np.ndarray:
        """Upsert devices by token fingerprint; returns device indices."""
        fp_lo = np.ascontiguousarray(fp_lo, np.uint64)
        fp_hi = np.ascontiguousarray(fp_hi, np.uint64)
        n = len(fp_lo)
        with self._lock:
            if dev_idx is None:
                dev_idx = np.arange(self.n_devices, self.n_devices + n, dtype=np.int32)
            dev_idx = np.ascontiguousarray(dev_idx, np.int32)
            if n and int(dev_idx.max()) >= self.cfg.max_devices:
                raise ValueError("device capacity exceeded (EngineConfig.max_devices)")
            slots = np.empty(n, np.int64)
            failed = native().sw_reg_build(_p(self.reg_lo), _p(self.reg_hi), _p(self.reg_val), self.cfg.reg_slots - 1,
                                           _p(fp_lo), _p(fp_hi), _p(dev_idx), n, _p(slots))
            if failed:
                raise RuntimeError("registry table full")
            self.dev_slot[dev_idx] = slots
            self.n_devices = max(self.n_devices, int(dev_idx.max()) + 1 if n else 0)
            if dev_type is not None:
                self.dev_type[dev_idx] = np.asarray(dev_type, np.int32)
                self._dirty_devices(dev_idx)
            self._dirty_registry(slots)
            return dev_idx

    def packed_registry(self, slots: np.ndarray) -> np.ndarray:
        """SwRegSlot rows for the given slots: fingerprint, device and *active* assignment."""
        rows = np.zeros(len(slots), REG_SLOT)
        rows["lo"] = self.reg_lo[slots]
        rows["hi"] = self.reg_hi[slots]
        dev = self.reg_val[slots]
        rows["dev"] = dev
        asg = np.where(dev >= 0, self.dev_asg[np.maximum(dev, 0)], -1)
        ok = (asg >= 0) & (self.asg_active[np.maximum(asg, 0)] > 0)
        rows["asg"] = np.where(ok, asg, -1)
        return rows

    def lookup_device(self, fp_lo: int, fp_hi: int) -> int:
        return int(native().sw_reg_find(_p(self.reg_lo), _p(self.reg_hi), _p(self.reg_val), self.cfg.reg_slots - 1,
                                        fp_lo, fp_hi))

    def set_assignments(self, asg_idx, dev_idx, customer=None, area=None, asset=None, active=None):
        """Create/update assignments and make them the device's active assignment when active."""
        asg_idx = np.atleast_1d(np.asarray(asg_idx, np.int32))
        dev_idx = np.atleast_1d(np.asarray(dev_idx, np.int32))
        n = len(asg_idx)
        if n and int(asg_idx.max()) >= self.cfg.max_assignments:
            raise ValueError("assignment capacity exceeded (EngineConfig.max_assignments)")

        def col(v, fill):
            return np.full(n, fill, np.int32) if v is None else np.broadcast_to(np.asarray(v, np.int32), (n,))

        act = np.ones(n, np.uint8) if active is None else np.broadcast_to(np.asarray(active, np.uint8), (n,))
        with self._lock:
            self._ctx_version += 1
            self.asg_device[asg_idx] = dev_idx
            self.asg_customer[asg_idx] = col(customer, -1)
            self.asg_area[asg_idx] = col(area, -1)
            self.asg_asset[asg_idx] = col(asset, -1)
            self.asg_active[asg_idx] = act
            on = act.astype(bool)
            self.dev_asg[dev_idx[on]] = asg_idx[on]
            # ending an assignment releases the device
            off_dev = dev_idx[~on]
            cur = self.dev_asg[off_dev]
            self.dev_asg[off_dev] = np.where(cur == asg_idx[~on], -1, cur)
            self.n_assignments = max(self.n_assignments, int(asg_idx.max()) + 1 if n else 0)
            self._dirty_assignments(asg_idx)
            self._dirty_devices(dev_idx)

    # ------------------------------------------------------------------ zones / rules
    def set_zone_rules(self, zones: list[Zone], tests: list[ZoneTest]):
        with self._lock:
            self.zones = list(zones)
            self.tests = list(tests)
            for t in tests:
                self.names[hash64(t.alert_type)] = t.alert_type
            self._zones_changed()

    def _zones_changed(self):
        pass

    def zone_arrays(self):
        """Flattened zone polygons: vtx [2*V] f64, off [Z+1] i32, bbox [4*Z] f64, tests ZONE_TEST[T]."""
        from ..models.columnar import ZONE_TEST

        idx = {z.token: i for i, z in enumerate(self.zones)}
        off = [0]
        vtx = []
        bbox = []
        for z in self.zones:
            v = np.asarray(z.vertices, np.float64).reshape(-1, 2)
            vtx.append(v.ravel())
            off.append(off[-1] + len(v))
            bbox.extend([v[:, 0].min(), v[:, 1].min(), v[:, 0].max(), v[:, 1].max()])
        tests = np.zeros(len(self.tests), ZONE_TEST)
        hashes = np.zeros(len(self.tests), np.uint64)
        for i, t in enumerate(self.tests):
            if t.zone_token not in idx:
                raise KeyError(f"zone test references unknown zone {t.zone_token!r}")
            tests[i] = (idx[t.zone_token], 0 if t.condition == "inside" else 1, -1, int(t.alert_level))
            hashes[i] = hash64(t.alert_type)
        return (np.concatenate(vtx) if vtx else np.zeros(2, np.float64), np.asarray(off, np.int32),
                np.asarray(bbox if bbox else [0.0] * 4, np.float64), tests, hashes)

    # ------------------------------------------------------------------ names
    def learn_names(self, refs: np.ndarray, raw: np.ndarray):
        """Record strings for newly seen name/type hashes (from this rank's raw batch)."""
        new = {}
        for r in refs:
            h = int(r["hash"])
            if h not in self.names:
                s = bytes(raw[int(r["off"]):int(r["off"]) + int(r["len"])]).decode("utf-8", "replace")
                self.names[h] = s
                new[h] = s
        return new

    def name_of(self, h: int) -> str | None:
        return self.names.get(int(h))

    def presence_due(self, now_ms: int) -> bool:
        if not self.presence_enabled or self.cfg.presence_missing_ms <= 0:
            return False
        if self._last_presence_check is None or now_ms - self._last_presence_check >= self.cfg.presence_check_ms:
            self._last_presence_check = now_ms
            return True
        return False

    def step_framed(self, batch, now_ms: int, presence: bool | None = None) -> StepResult:
        """Step a :class:`~sitewhere_amd.pipeline.bus_io.RawBatch` (a raw-payload record read from the
        bus, possibly in place).  Host engines rebuild the offsets; the MI355X engine overrides this
        to DMA the payload and its varint lengths straight from the record."""
        return self.step(np.asarray(batch.payload)[:batch.payload_bytes], batch.offsets(), now_ms, presence=presence)

    # ------------------------------------------------------------------ overlapped (lagged) steps
    # A service tenant feeds batches one at a time from its raw-payload consumer.  On the MI355X the
    # H2D of batch k overlaps the compute of batch k-1 and the D2H of k-1's rows overlaps the compute
    # of batch k, so a submitted batch's result comes back on a LATER submission (or on
    # ``drain_framed``), always in submission order.  Host engines keep a one-deep lag -- they run a
    # batch when the next arrives -- so callers are written (and tested on CPU) once.  The batch's
    # memory (a topic record read in place) must stay valid until its result is returned.
    def submit_framed(self, batch, now_ms: int, token=None, presence: bool | None = None) -> list:
        """Enqueue one raw batch; returns ``[(token, StepResult)]`` of the submissions completed."""
        done = self.drain_framed()
        self._lagged = (batch, now_ms, token, presence)
        return done

    def drain_framed(self) -> list:
        """Complete every submitted batch; ``[(token, StepResult)]`` in submission order."""
        lag = getattr(self, "_lagged", None)
        if lag is None:
            return []
        self._lagged = None
        batch, now_ms, token, presence = lag
        return [(token, self.step_framed(batch, now_ms, presence))]

    def carry_count(self) -> int:
        """Records deferred to the next exchange (host-known; multi-rank engines)."""
        return 0

    def should_stall(self) -> bool:
        """Multi-rank drivers feed an empty round (exchange only) instead of a new batch while this
        is true: skewed keys then slow the input down instead of losing records at ``carry_cap``.
        Every rank still runs one round per iteration, so the collective stays in step."""
        return self.world > 1 and self.carry_count() > self.cfg.carry_high

    @property
    def framed_pending(self) -> int:
        """Submitted batches whose results have not been returned yet."""
        return 0 if getattr(self, "_lagged", None) is None else 1

    # ------------------------------------------------------------------ store-backed dedup filter
    # Engines implement four primitives over their filter (pipeline/dedup_filter.py layout):
    # _ff_meta_get / _ff_meta_set (meta words), _ff_add (ids into one generation, not counted),
    # _ff_clear (one generation).
    @property
    def filter_on(self) -> bool:
        return bool(getattr(self.cfg, "dedup_filter_ids", 0))

    def filter_seed_begin(self):
        """Start a warm start from the durable store (:meth:`filter_seed`)."""
        m = self._ff_meta_get() if self.filter_on else None
        self._seed = [int(m[0]), int(m[6]), 0] if m is not None else None

    def filter_seed(self, hashes) -> int:
        """Warm start from the durable store: ``hashes`` are stored alternate ids, NEWEST FIRST (call
        once per chunk, in that order, after :meth:`filter_seed_begin`).  The newest fill the live
        generation, older ones the generations before it (each up to its ids), as if the engine had
        persisted them; what no generation can take is older than the filter remembers -- retention
        by rows keeps it out of the store anyway.  Returns the ids added."""
        if not self.filter_on:
            return 0
        if getattr(self, "_seed", None) is None:
            self.filter_seed_begin()
        h = np.asarray(hashes, np.uint64)
        h = h[h != 0]
        m = self._ff_meta_get()
        G, C = int(m[3]), int(m[2])
        g, k, filled = self._seed
        i = added = 0
        while i < len(h) and filled < G:
            take = h[i:i + max(0, C - k)]
            if len(take):
                self._ff_add(take, g)
                k += len(take)
                i += len(take)
                added += len(take)
                if g == int(m[0]):
                    m[6] = k
            if k >= C:                               # this generation is full: the one before it
                filled += 1
                g, k = (g - 1) % G, 0
        self._seed = [g, k, filled]
        self._ff_meta_set(m)
        return added

    def filter_state(self) -> dict:
        """The filter's live generation, rotations, ids taken, probe drops (``dedup_filter.filter_state``)."""
        if not self.filter_on:
            return {}
        from .dedup_filter import filter_state
        return filter_state(self._ff_meta_get())

    # ------------------------------------------------------------------ hot-store queries
    def query_store(self, event_type: int, asg_idx, start: int | None = None, end: int | None = None,
                    page_number: int = 1, page_size: int = 100):
        """Events of one type for a set of assignment indices in a date range, newest first (ties:
        latest event id first), straight from this shard's event ring -- the hot half of
        ``DeviceEventManagement.list*ForIndex``.  Returns (total, page columns dict, page event ids)."""
        raise NotImplementedError

    @staticmethod
    def _window(page_number: int, page_size: int, total: int) -> tuple[int, int]:
        if page_size <= 0:
            return 0, total
        lo = (max(1, page_number) - 1) * page_size
        return min(lo, total), min(lo + page_size, total)

    def _row_seq(self, rows, cursor: int):
        """Store sequence of ring rows (works on numpy and torch integer arrays)."""
        cap = self.cfg.store_cap
        if cursor <= cap:
            return rows
        return (cursor - cap) + (rows - (cursor % cap)) % cap

    # ------------------------------------------------------------------ durable blocks
    def encode_block(self, now_ms: int, res: StepResult | None = None, slot: int | None = None,
                     boot: int = 0) -> np.ndarray:
        """Durable block (``persistence/segments.py``) of a step: encoded and sealed on the host from
        the step's rows, persisted records, string refs and raw batch (the whole event: alternate
        ids, alert messages, metadata).  The MI355X engine overrides this with its GPU encoder
        (same bytes)."""
        from ..persistence.segments import encode_block, seal
        ix = self.cfg.block_index
        blk = encode_block(res.out if res.out is not None else np.zeros(0, OUT_REC), res.prec, res.pspans, res.raw,
                           index=ix, ctx=self.ctx_table() if ix else None)
        res.raw = None
        seal(blk, res.first_seq, now_ms, boot, self.rank, self.world)
        return blk

    def ctx_table(self) -> np.ndarray:
        """Assignment context by assignment index, int32 [max_assignments, 4] = (device, customer,
        area, asset): what the block index trailer keys its context dimensions by (the MI355X engine
        reads its HBM copy, ``asg_ctx``)."""
        tab = self.__dict__.get("_ctx_tab")
        if tab is None or tab[0] != self._ctx_version:
            t = np.ascontiguousarray(np.stack([self.asg_device, self.asg_customer, self.asg_area, self.asg_asset], 1),
                                     np.int32)
            tab = self._ctx_tab = (self._ctx_version, t)
        return tab[1]

    _ctx_version = 0

    def ctx_key_spaces(self) -> np.ndarray:
        """Per context dimension (customer, area, asset) the block index's key space: (max context
        id + 1) << 3, 0 when no assignment has one, -1 when ids reach the indexed range's end
        (swindex.h SIX_CTX_MAX: that dimension goes unindexed)."""
        ks = self.__dict__.get("_ctx_keys")
        if ks is None or ks[0] != self._ctx_version:
            out = np.zeros(3, np.int32)
            for d, col in enumerate((self.asg_customer, self.asg_area, self.asg_asset)):
                m = int(col.max()) if len(col) else -1
                out[d] = -1 if m >= 8192 else ((m + 1) << 3 if m >= 0 else 0)
            ks = self._ctx_keys = (self._ctx_version, out)
        return ks[1]

    # ------------------------------------------------------------------ checkpoint / resume
    kind = "base"
    dedup_valid_from = 0          # store sequence from which the dedup window saw every row's id

    def checkpoint_state(self, include_store: bool = False) -> dict:
        """Engine tables to snapshot (name -> numpy array); see ``pipeline/checkpoint.py``."""
        raise NotImplementedError

    def restore_state(self, arrays: dict, include_store: bool):
        raise NotImplementedError

    def save_checkpoint(self, path: str, include_store: bool = False, extra: dict | None = None) -> int:
        from .checkpoint import save_engine
        return save_engine(self, path, include_store, extra)

    def load_checkpoint(self, path: str) -> dict:
        from .checkpoint import load_engine
        return load_engine(self, path)

    @staticmethod
    def stats_dict(arr) -> dict:
        return {n: int(arr[i]) for i, n in enumerate(STAT_NAMES)}
