"""MI355X inbound tenant engine: the fused micro-batch pipeline behind service-inbound-processing.

Replaces the per-event path of the reference (``DecodedEventsConsumer.java:79-204`` ->
``InboundPayloadProcessingLogic.java:101-218`` -> ``UnaryEventStorageStrategy.java:53-90`` ->
``KafkaEventPersistenceTriggers`` -> ``PersistedEventsConsumer`` / ``OutboundPayloadEnrichmentLogic``)
with one engine step per batch of raw payloads:

  raw batch record (``<tenant>event-source-raw-payloads``, written by event sources configured with
  ``"forward": "raw"``) -> :class:`GpuInboundEngine` (decode, registry lookup + assignment validation,
  alternate-id dedup, persist into the HBM event ring, enrichment, device-state merge, zone rules,
  presence) -> enriched events on ``inbound-enriched-events`` + bulk insert into event management.

The registry mirror is kept current from the device-model change feed (``device-model-updates``)
that device management publishes on every mutation, so no per-event RPC happens.  Messages the
engine does not persist but that need a control-plane decision (unregistered devices, registration,
acknowledgements, streams) take a slow path: the batch is re-decoded on the host and those messages
are routed exactly like the reference routes them (unregistered / registration topics).

``device`` config: ``"gpu"`` (fail loudly without a GPU), ``"cpu"`` (the native multi-threaded C++ engine,
``pipeline/native_engine.py``), ``"oracle"`` (the Python reference engine) or ``"auto"`` (GPU if present).
"""
from __future__ import annotations

import json
import queue
import threading
import time

import numpy as np

from ..models.columnar import (EV_ALERT, EV_LOCATION, EV_MEASUREMENT, EV_STATE_CHANGE, NO_NAME, OUT_REC,
                               ST_CONTROL, ST_UNASSIGNED, ST_UNREGISTERED)
from ..persistence.columnar import encode_batch, frame_batch
from ..models.domain import (AlertLevel, AlertSource, DeviceAlert, DeviceAssignmentStatus, DeviceLocation,
                             DeviceMeasurement, DeviceStateChange, now_ms)
from ..pipeline.config import EngineConfig
from ..pipeline.engine_base import Zone, ZoneTest
from ..pipeline.bus_io import MultiRawBatch, RawBatch, parse_raw_batch
from ..pipeline.fleet import fingerprint_str, pack_messages
from ..rpc import codec
from ..utils import IndexMap, retain_large_allocations, tune_gc_for_streaming
from ..runtime.consumers import BusConsumer, RetryFrom
from ..bus import payloads
from .event_sources import RAW_PAYLOADS, ProtobufDecoder
from .inbound_processing import InboundProcessingTenantEngine

_LEVELS = [AlertLevel.Info, AlertLevel.Warning, AlertLevel.Error, AlertLevel.Critical]
ENRICHED_BATCHES = "inbound-enriched-batches"     # columnar enriched output (publishEnriched = "batches")


def unpack_raw_batch(value: bytes):
    """A raw-payload record value -> (raw uint8 with 64 bytes of padding, offs uint32[n+1])."""
    rb = parse_raw_batch(value)
    return np.array(rb.payload), rb.offsets()


class _Stepped:
    """A raw batch the engine has stepped, with the storage stages it has completed.  The raw bytes
    are not kept: rejected messages are routed (``_route``) as soon as the step completes."""
    __slots__ = ("key", "res", "now", "batch", "stored", "published", "routed", "queued", "payload", "events",
                 "detach", "hold", "commit", "trace", "routed_recs", "token", "first")

    def __init__(self, key, res, now, batch, first=None):
        self.key, self.res, self.now, self.batch = key, res, now, batch
        # key = (topic, partition, offset) of the batch's last raw record; first = offset of its first
        # (records coalesced into one step, see _process_raw)
        self.first = first if first is not None or key is None else key[2]
        self.stored = self.published = self.routed = self.queued = False
        self.payload = self.events = None
        self.detach, self.hold, self.commit = False, None, None
        self.trace = None
        self.routed_recs = None                 # the rejects, routed while the raw record was readable
        self.token = None                       # durable storage: the store's token of the block


class GpuInboundTenantEngine(InboundProcessingTenantEngine):
    """Raw protobuf batches run through the fused engine; decoded requests that did not come through
    the raw path (JSON sources, reprocessed events) keep the inherited per-event path."""

    def tenant_initialize(self, monitor):
        super().tenant_initialize(monitor)      # decoded / persisted consumers, near caches, meters
        cfg = self.config
        ms, t = self.ms, self.tenant.token
        n = ms.instance.naming
        self.t_enriched = n.inbound_enriched_events(t)
        self.t_unregistered = n.unregistered_device_events(t)
        self.t_registration = n.device_registration_events(t)
        self.t_decoded = n.decoded_events(t)
        self.t_failed_decode = n.failed_decode_events(t)
        self.routed_payloads = 0                # payloads the slow path parsed (per payload, not per batch)
        self.recheck_duplicates = 0             # filter rechecks whose hash the durable store holds (replays)
        self.recheck_false_positives = 0        # filter rechecks the store did not know (host path)
        self._fp_win = [0, 0]                   # false positives / engine payloads since the last check
        self.dedup_sizing_report: dict = {}
        self.t_enriched_batches = n.tenant_prefix(t) + ENRICHED_BATCHES
        # objects: per-event host objects; columnar: row batches; durable: encoded blocks (GPU-encoded
        # on the MI355X) to a durable segment store, offsets committed once on disk
        self.storage = cfg.get("storage", "objects")            # objects | columnar | durable
        self.publish = cfg.get("publishEnriched", "events")     # events | batches | none
        self._asg_dirty: set[int] = set()
        self._names_sent = 0
        self._names_known = -1
        ecfg = EngineConfig.small(**{k: int(v) for k, v in cfg.get("capacity", {}).items()}) \
            if cfg.get("sizing", "small") == "small" else EngineConfig(**cfg.get("capacity", {}))
        ecfg.presence_missing_ms = int(cfg.get("presenceMissingMs", ecfg.presence_missing_ms))
        ecfg.presence_check_ms = int(cfg.get("presenceCheckMs", ecfg.presence_check_ms))
        self.engine_cfg = ecfg
        self.engine = self._make_engine(cfg.get("device", "auto"), ecfg)
        if self.storage in ("columnar", "durable") and cfg.get("retainHostAllocations", True):
            retain_large_allocations()          # multi-MB columnar batches per step: no fresh mmaps
        self.dev_index, self.asg_index = IndexMap(), IndexMap()
        self.customers, self.areas, self.assets = IndexMap(), IndexMap(), IndexMap()
        self._asg_entities: dict[int, object] = {}
        self._dev_tokens: dict[int, str] = {}
        self._dev_types: dict[int, str] = {}
        self._nid2name: dict[int, str] = {}
        self._lock = threading.RLock()
        self.boot = f"{int(time.time() * 1000):x}"
        self._set_boot(self.boot)
        self.zone_tests = [ZoneTest(z["zoneToken"], z.get("condition", "inside"), z.get("alertType", "zone.alert"),
                                    int(z.get("alertLevel", 1)), z.get("alertMessage", ""))
                           for z in cfg.get("zoneTests", [])]
        # checkpoint / resume: {"path": ..., "everyBatches": N, "includeStore": false}.
        # With a checkpoint the raw consumer commits only the offsets a snapshot on disk covers.
        ck = cfg.get("checkpoint") or {}
        self.ckpt_path = ck.get("path") or None      # already [[tenant.token]]-substituted
        self.ckpt_every = int(ck.get("everyBatches", 64))
        self.ckpt_store = bool(ck.get("includeStore", False))
        self._ckpt_offsets: dict[tuple[str, int], int] = {}
        self._since_ckpt = 0
        self.checkpoints = 0
        # Host-side storage of a step's rows (columnar encode, event-management RPC, enriched publish)
        # runs on a store thread, overlapped with the next engine step.  Raw-topic offsets are then
        # committed by that thread once a batch is stored (at-least-once holds); with a checkpoint
        # the snapshot owns the commits.
        self.async_store = bool(cfg.get("asyncStore", self.storage in ("columnar", "durable")))
        # opt-in: columnar payloads framed around the rows in the engine's pinned row buffers (no
        # host copy).  The enriched-batch topic and the columnar store then hold those buffers until
        # their retention drops them, so it pays only when both windows fit the engine's buffer pool
        # (batches stick to one topic partition for that, _batch_partition): +26-35% at 1M-payload
        # batches with an 8-batch store window, but with the store's default window (every batch
        # kept) the pool runs dry and each step pays a fresh pinned allocation
        # (profiles/r2_tenant_zcrows)
        self.zero_copy_rows = bool(cfg.get("zeroCopyRows", False))
        self._sticky_part: int | None = None
        self.zc_framed = self.zc_copied = 0
        self._store_q: queue.Queue = queue.Queue(maxsize=2)
        # durable storage: stored batches whose block is not on disk yet, in order -- their raw
        # offsets commit (and the batch leaves _stepped) once the store's durable token passes theirs,
        # so the store thread never sits in an fdatasync
        from collections import deque
        self._durable_wait: deque = deque()
        self._durable_lock = threading.Lock()
        self._store_thread = None
        self._store_error = None
        # Overlapped engine steps (``overlapSteps``, default on for MI355X columnar tenants): a raw
        # batch is submitted to the engine and completes when the next one is submitted, so its H2D
        # and row D2H overlap the neighbouring batches' compute (``EngineBase.submit_framed``).  A
        # submitted batch's record stays readable through a retention hold of this engine until its
        # result is back; the pipeline is drained whenever the raw topic has nothing more queued.
        self.overlap = bool(cfg.get("overlapSteps", self.async_store and self.engine_kind == "gpu"))
        # step raw records that are already waiting in one partition together (overlapped steps only)
        self.coalesce = bool(cfg.get("coalesceRaw", True))
        self._order_lock = threading.Lock()    # engine submit/drain + completion hand-off, in step order
        self._holds: dict[tuple, dict] = {}    # (topic, partition) -> {offset: in-flight batches}
        self._hold_lock = threading.Lock()      # the consumer and the reject router both release holds
        # SW_TENANT_TRACE=1: per-batch timestamps (submit, submitted, completed, store start, payload,
        # stored, published) for the tenant-path bench's breakdown
        import os
        self.trace = [] if os.environ.get("SW_TENANT_TRACE") == "1" else None
        # Replay safety.  engine.step is not idempotent (cursor, event ids, dedup table and device
        # state advance), so a raw record is stepped at most once per engine lifetime: its StepResult
        # stays in ``_stepped`` until every storage stage succeeded, and a re-read record (consumer
        # retry / rewind) reuses it and retries only the stages still missing.  ``_stored_hw`` is,
        # per partition, the offset below which every record is fully stored (stores run in step
        # order), so a replayed prefix is skipped outright.
        self._stepped: dict[tuple, _Stepped] = {}
        self._stored_hw: dict[tuple, int] = {}
        self.replayed_batches = 0
        self.dead_lettered = 0                 # raw records that failed validation before a step
        # the consumer itself never dead-letters: a stepped batch cannot be re-stepped, only its
        # storage retried; records that fail validation before a step are dead-lettered by the
        # handler (_dead_letter_raw)
        self.raw_consumer = BusConsumer(self, "raw-payload-consumers", [n.tenant_prefix(t) + RAW_PAYLOADS],
                                        self._process_raw, max_records=16, max_attempts=None,
                                        idle=self._on_idle, views=True,
                                        auto_commit=self.ckpt_path is None and not self.async_store)
        self.persisted_events = self.create_meter("persistedEvents")
        self.step_timer = self.create_timer("engineStep")
        self.store_timer = self.create_timer("columnarStore")       # payload build + event-management call
        self.publish_timer = self.create_timer("enrichedPublish")
        self.recheck_timer = self.create_timer("filterRecheck")       # durable-store lookup of rechecks
        self.api = {"InboundProcessing": GpuInboundApi(self)}

    def _make_engine(self, device: str, ecfg: EngineConfig):
        want_gpu = device == "gpu"
        if device in ("gpu", "auto"):
            try:
                import torch
                if torch.cuda.is_available():
                    import os
                    from ..pipeline.gpu_engine import GpuInboundEngine
                    self.engine_kind = "gpu"
                    # one inbound-processing replica per GPU: the replica's device comes from its
                    # configuration, SITEWHERE_GPU_DEVICE, or the launcher's LOCAL_RANK
                    idx = self.config.get("gpuDevice", os.environ.get("SITEWHERE_GPU_DEVICE",
                                                                      os.environ.get("LOCAL_RANK", 0)))
                    self.gpu_device = int(idx) % torch.cuda.device_count()
                    return GpuInboundEngine(ecfg, device=f"cuda:{self.gpu_device}")
            except Exception:
                if want_gpu:
                    raise
            if want_gpu:
                raise RuntimeError("inbound-processing configured with device=gpu but no GPU is available")
        self.engine_kind = "cpu"
        if device == "oracle":
            from ..pipeline.cpu_engine import CpuInboundEngine
            return CpuInboundEngine(ecfg)
        from ..pipeline.native_engine import NativeCpuEngine
        return NativeCpuEngine(ecfg, threads=int(self.config.get("cpuThreads", 0)) or None)

    def _set_boot(self, boot: str):
        """Engine incarnation: event ids are ``<boot>-<id>``; durable blocks carry it numerically."""
        from ..persistence.segments import boot_id
        self.boot = boot
        self.block_boot = boot_id(boot)
        # durable: the block is what is stored; objects: the block is where each row's strings are
        # (alternate id, alert message, metadata) when the rows become event objects (_to_events)
        if self.storage in ("durable", "objects") and hasattr(self.engine, "encode_blocks"):
            self.engine.encode_blocks = True            # MI355X: blocks encoded on the GPU per step
            self.engine.block_boot = self.block_boot

    def _ensure_block(self, res, now: int):
        """Host engines encode the step's block on the completing thread (their event ring is
        overwritten by later steps)."""
        if self.storage in ("durable", "objects") and res is not None and res.block is None:
            res.block = self.engine.encode_block(now, res, boot=self.block_boot)

    # ---------------------------------------------------------------- registry mirror
    def _dm(self):
        return self.ms.api("DeviceManagement", self.tenant.token)

    def _em(self):
        return self.ms.api("DeviceEventManagement", self.tenant.token)

    def load_model(self):
        """Full registry load (device management list APIs), then the change feed keeps it current.
        One engine call for all devices and one for all assignments: per entity, a 1M-device tenant
        paid a table upload (and its stream sync) per device and per assignment at every start."""
        dm = self._dm()
        devs = dm.list_devices({"pageSize": 0}).results
        asgs = dm.list_device_assignments({"pageSize": 0}).results
        with self._lock:
            if devs:
                di = np.array([self.dev_index.get(d.id) for d in devs], np.int32)
                fps = np.array([fingerprint_str(d.token) for d in devs], np.uint64).reshape(-1, 2)
                self.engine.register_devices(np.ascontiguousarray(fps[:, 0]), np.ascontiguousarray(fps[:, 1]), di)
                for d, i in zip(devs, di.tolist()):
                    self._dev_tokens[i] = d.token
                    self._dev_types[i] = d.device_type_id
            if asgs:
                # in list order, as the per-entity upserts were: the last active assignment of a
                # device wins, and a released one clears the device only while it is current
                ai = [self.asg_index.get(a.id) for a in asgs]
                dv = [self.dev_index.get(a.device_id) for a in asgs]
                self.engine.set_assignments(ai, dv, customer=[self.customers.get(a.customer_id) for a in asgs],
                                            area=[self.areas.get(a.area_id) for a in asgs],
                                            asset=[self.assets.get(a.asset_id) for a in asgs],
                                            active=[0 if a.status == DeviceAssignmentStatus.Released else 1
                                                    for a in asgs])
                for a, i in zip(asgs, ai):
                    self._asg_entities[i] = a
                    self._asg_dirty.add(i)
        self._load_zones()

    def _load_zones(self):
        if not self.zone_tests:
            return
        dm = self._dm()
        zones = []
        for tok in sorted({zt.zone_token for zt in self.zone_tests}):
            z = dm.get_zone_by_token(tok)
            if z is not None:
                zones.append(Zone(z.token, [(p["latitude"], p["longitude"]) if isinstance(p, dict)
                                            else (p.latitude, p.longitude) for p in z.bounds]))
        known = {z.token for z in zones}
        self.engine.set_zone_rules(zones, [zt for zt in self.zone_tests if zt.zone_token in known])

    def _upsert_device(self, d):
        with self._lock:
            di = self.dev_index.get(d.id)
            lo, hi = fingerprint_str(d.token)
            self.engine.register_devices(np.array([lo], np.uint64), np.array([hi], np.uint64), np.array([di], np.int32))
            self._dev_tokens[di] = d.token
            self._dev_types[di] = d.device_type_id

    def _upsert_assignment(self, a):
        with self._lock:
            di = self.dev_index.get(a.device_id)
            known = int(self.engine.dev_slot[di]) >= 0
        d = None
        if not known:
            # the assignment's event came before its device's (the change feed does not order them):
            # register the device now, or its payloads route as unregistered until the device event
            # arrives although the assignment is active.  Fetched before taking the engine lock (a
            # slow device-management call must not stall the store path's dictionary deltas).
            try:
                d = self._dm().get_device(a.device_id)
            except Exception as e:      # noqa: BLE001 -- the device event registers it later
                self.logger.warning("device %s of assignment %s not registered yet (%s): its device event will",
                                    a.device_id, a.id, e)
        with self._lock:
            ai = self.asg_index.get(a.id)
            if d is not None and int(self.engine.dev_slot[di]) < 0:
                self._upsert_device(d)
            active = a.status != DeviceAssignmentStatus.Released
            self.engine.set_assignments([ai], [di], customer=[self.customers.get(a.customer_id)],
                                        area=[self.areas.get(a.area_id)], asset=[self.assets.get(a.asset_id)],
                                        active=[1 if active else 0])
            self._asg_entities[ai] = a
            self._asg_dirty.add(ai)

    def _upsert_devices(self, devs):
        """Many devices in one registry upload (a bulk create's change-feed records)."""
        with self._lock:
            di = np.array([self.dev_index.get(d.id) for d in devs], np.int32)
            fps = np.array([fingerprint_str(d.token) for d in devs], np.uint64).reshape(-1, 2)
            self.engine.register_devices(np.ascontiguousarray(fps[:, 0]), np.ascontiguousarray(fps[:, 1]), di)
            for d, i in zip(devs, di.tolist()):
                self._dev_tokens[i] = d.token
                self._dev_types[i] = d.device_type_id

    def _upsert_assignments(self, asgs):
        """Many assignments in one engine call, in feed order (the last one of a device wins)."""
        with self._lock:
            missing = [a.device_id for a in asgs if int(self.engine.dev_slot[self.dev_index.get(a.device_id)]) < 0]
        if missing:                              # rare: their devices' records have not arrived yet
            for a in asgs:
                self._upsert_assignment(a)
            return
        with self._lock:
            ai = [self.asg_index.get(a.id) for a in asgs]
            self.engine.set_assignments(ai, [self.dev_index.get(a.device_id) for a in asgs],
                                        customer=[self.customers.get(a.customer_id) for a in asgs],
                                        area=[self.areas.get(a.area_id) for a in asgs],
                                        asset=[self.assets.get(a.asset_id) for a in asgs],
                                        active=[0 if a.status == DeviceAssignmentStatus.Released else 1 for a in asgs])
            for a, i in zip(asgs, ai):
                self._asg_entities[i] = a
                self._asg_dirty.add(i)

    def _apply_model_changes(self, changes):
        super()._apply_model_changes(changes)   # near-cache invalidation for the per-event path
        # runs of device creates / updates and of assignment creates / updates are applied in one
        # engine call each (a bulk provisioning publishes thousands at once); order is kept
        run_kind, run = None, []

        def flush():
            if run_kind == "device":
                self._upsert_devices(run) if len(run) > 1 else self._upsert_device(run[0])
            elif run_kind == "assignment":
                self._upsert_assignments(run) if len(run) > 1 else self._upsert_assignment(run[0])
            run.clear()

        for kind, e in changes:
            k = ("device" if kind in ("device.created", "device.updated")
                 else "assignment" if kind in ("assignment.created", "assignment.imported", "assignment.updated",
                                               "assignment.ended")
                 else None)
            if k != run_kind:
                flush()
                run_kind = k
            if k is not None:
                run.append(e)
                continue
            if kind == "device.deleted":
                with self._lock:
                    # tombstone: the fingerprint keeps its slot but resolves to no active assignment
                    di = self.dev_index.get(e.id)
                    self.engine.dev_asg[di] = -1
                    self.engine._dirty_devices(np.array([di], np.int32))
            elif kind == "assignment.deleted":
                e.status = DeviceAssignmentStatus.Released
                self._upsert_assignment(e)
            elif kind.startswith("zone."):
                self._load_zones()
        flush()
        if self._store_thread is not None or self.storage == "durable":
            self._prime_dictionary()            # a bulk import: its dictionary ahead of the blocks

    # ---------------------------------------------------------------- lifecycle
    def tenant_start(self, monitor):
        self.restore_checkpoint()
        self.load_model()
        super().tenant_start(monitor)           # model-update, decoded and persisted consumers
        self._resume_from_store()
        self._prime_dictionary()
        if self.config.get("tuneGc", False):
            tune_gc_for_streaming()             # after the registry and dictionary are built
        self.check_dedup_sizing()
        bus = self.ms.instance.bus
        if self.config.get("rawBackpressure", True) and hasattr(bus, "protect"):
            # raw batches this engine has not committed are never dropped by retention; event
            # sources wait for room instead (EventBus.protect)
            for t in self.raw_consumer.topics:
                bus.protect(self.raw_consumer.group, t, float(self.config.get("rawBackpressureWaitS", 60)))
        if self.async_store:
            self._store_thread = threading.Thread(target=self._store_loop, daemon=True,
                                                  name=f"engine-store-{self.tenant.token}")
            self._store_thread.start()
        self.start_nested_component(self.raw_consumer, monitor, require=True)

    def tenant_stop(self, monitor):
        self.raw_consumer.lifecycle_stop(monitor)
        bus = self.ms.instance.bus
        if hasattr(bus, "unprotect"):
            for t in self.raw_consumer.topics:
                bus.unprotect(self.raw_consumer.group, t)
        if self._store_thread is not None:
            self.flush()
            self._store_q.put(None)
            self._store_thread.join(10)
            self._store_thread = None
        pool = self.__dict__.pop("_route_pool", None)
        if pool is not None:
            pool.shutdown(wait=True)
        if self.ckpt_path and self._since_ckpt:
            if self._store_error is None and not self._stepped:
                self.checkpoint()
            else:               # the next start replays from the last good checkpoint instead
                self.logger.error("not checkpointing on stop: %d stepped batches are not stored", len(self._stepped))
        super().tenant_stop(monitor)

    # ---------------------------------------------------------------- checkpoint / resume
    def checkpoint(self):
        """Snapshot the shard + the raw-topic offsets it covers, then commit those offsets."""
        import os
        self.flush()            # every batch the snapshot covers must be stored before its offset commits
        self._raise_store_error()
        if self._stepped:
            # the snapshot would cover engine state whose rows were never stored: committing its
            # offsets would lose them.  The raw consumer re-reads and re-stores first.
            raise RuntimeError(f"refusing to checkpoint: {len(self._stepped)} stepped batches not stored")
        with self._lock:
            extra = {"boot": self.boot, "offsets": [[t, p, o] for (t, p), o in self._ckpt_offsets.items()],
                     "dev_index": self.dev_index.ids, "asg_index": self.asg_index.ids,
                     "customers": self.customers.ids, "areas": self.areas.ids, "assets": self.assets.ids}
            os.makedirs(os.path.dirname(os.path.abspath(self.ckpt_path)), exist_ok=True)
            self.engine.save_checkpoint(self.ckpt_path, include_store=self.ckpt_store, extra=extra)
            self._since_ckpt = 0
            self.checkpoints += 1
        bus = self.ms.instance.bus
        for (t, p), o in dict(self._ckpt_offsets).items():
            bus.commit(self.raw_consumer.group, t, p, o)

    def restore_checkpoint(self) -> bool:
        import os
        if not self.ckpt_path or not os.path.exists(self.ckpt_path):
            return False
        with self._lock:
            extra = self.engine.load_checkpoint(self.ckpt_path)
            self._set_boot(extra["boot"])
            for name in ("dev_index", "asg_index", "customers", "areas", "assets"):
                m = getattr(self, name)
                for key in extra[name]:
                    m.get(key)
            self._ckpt_offsets = {(t, int(p)): int(o) for t, p, o in extra["offsets"]}
        # the snapshot's offsets are authoritative: replay starts right after what it covers
        bus = self.ms.instance.bus
        for (t, p), o in self._ckpt_offsets.items():
            bus.commit(self.raw_consumer.group, t, p, o)
        self.logger.info("restored engine shard from %s (%d offsets)", self.ckpt_path, len(self._ckpt_offsets))
        return True

    # ---------------------------------------------------------------- data plane
    COALESCE_MAX_RECORDS = 16

    def _process_raw(self, recs):
        """Step the raw records of one poll.  Records of one partition that are already waiting are
        coalesced into one engine step (up to the engine's batch capacity): under load, small
        micro-batches then share one step's fixed cost; an idle partition still steps each record as
        it arrives (the event sources' latency bound holds)."""
        group = []                                      # [(record, parsed batch)] of one partition, consecutive
        resubmitted = set()
        pre = self._prevalidate(recs)

        def flush():
            if not group:
                return
            first_r, last_r = group[0][0], group[-1][0]
            view = isinstance(first_r.value, memoryview)
            batch = group[0][1] if len(group) == 1 else MultiRawBatch([b for _, b in group])
            commit = (last_r.topic, last_r.partition, last_r.offset + 1) \
                if self.async_store and not self.ckpt_path else None
            self.process_raw_batch(batch, now=last_r.timestamp or None, commit=commit,
                                   key=(last_r.topic, last_r.partition, last_r.offset), detach=view,
                                   hold=(first_r.topic, first_r.partition, first_r.offset) if view else None,
                                   first=first_r.offset)
            if self.ckpt_path:
                for r, _ in group:
                    self._ckpt_offsets[(r.topic, r.partition)] = r.offset + 1
                    self._since_ckpt += 1
                if self._since_ckpt >= self.ckpt_every:
                    self.checkpoint()
            group.clear()

        for ri, r in enumerate(recs):
            tp = (r.topic, r.partition)
            self._raise_store_error()                   # before any new step, never after
            if r.offset < self._stored_hw.get(tp, -1):
                continue                                # fully stored on an earlier read
            key = (r.topic, r.partition, r.offset)
            item = self._stepped.get(key)
            if item is not None:
                flush()
                if id(item) in resubmitted:
                    continue                            # a later record of a group already resubmitted
                resubmitted.add(id(item))
                if item.res is None:                    # still in the engine: complete it first
                    self._drain_engine()
                self.replayed_batches += 1
                t, p, o = item.key
                self._submit(item, (t, p, o + 1) if self.async_store and not self.ckpt_path else None)
                if self.ckpt_path:
                    self._ckpt_offsets[tp] = o + 1
                continue
            # r.value is a zero-copy view of the topic on the in-process bus: a pinned raw-batch
            # record is DMA'd to the MI355X in place.  The record timestamp is the batch's receive
            # time, so replay after a restore is deterministic.
            try:
                batch, err = pre[ri]
                if err is not None:
                    raise err
                if batch.n_msgs > self.engine_cfg.max_msgs:
                    raise ValueError(f"raw batch of {batch.n_msgs} payloads exceeds the engine's "
                                     f"max_msgs={self.engine_cfg.max_msgs}")
            except ValueError as e:
                # never stepped, so nothing to keep: a poison record is dead-lettered, not retried
                # forever (the unlimited retries below are only for stepped-but-unstored batches)
                flush()
                self._dead_letter_raw(r, e, (r.topic, r.partition, r.offset + 1)
                                      if self.async_store and not self.ckpt_path else None)
                if self.ckpt_path:
                    self._ckpt_offsets[tp] = r.offset + 1
                continue
            if group:
                g0, gl = group[0][0], group[-1][0]
                fits = (self.coalesce and self.overlap and batch.lens is not None
                        and all(b.lens is not None for _, b in group)
                        and (r.topic, r.partition) == (g0.topic, g0.partition) and r.offset == gl.offset + 1
                        and len(group) < self.COALESCE_MAX_RECORDS
                        and sum(b.n_msgs for _, b in group) + batch.n_msgs <= self.engine_cfg.max_msgs)
                if not fits:
                    flush()
            group.append((r, batch))
        flush()
        if recs and self.engine.framed_pending:
            last = recs[-1]
            end = getattr(self.ms.instance.bus, "end_offset", None)
            if end is None or end(last.topic, last.partition) <= last.offset + 1:
                self._drain_engine()                    # nothing more queued: complete the last batch

    def _prevalidate(self, recs) -> list:
        """(parsed batch, None) or (None, ValueError) per record: the framing of every record of a
        poll checked at once, on a small pool (the native length parse releases the interpreter),
        instead of one after another on the consumer thread that also drives the engine -- with
        alternate ids a 64K-payload record's lengths mix one- and two-byte varints and take ~0.1 ms
        to check, a quarter of that thread's time per step (profiles/r5_tenant)."""
        def one(r):
            try:
                b = parse_raw_batch(r.value)
                b.validate()
                return b, None
            except ValueError as e:
                return None, e
        if len(recs) < 2:
            return [one(r) for r in recs]
        pool = self.__dict__.get("_val_pool")
        if pool is None:
            from concurrent.futures import ThreadPoolExecutor
            pool = self._val_pool = ThreadPoolExecutor(4, thread_name_prefix="raw-validate")
        return list(pool.map(one, recs))

    def _dead_letter_raw(self, r, err, commit):
        """Park a raw record that cannot be stepped (corrupt framing, over-size batch) on
        ``<topic>.dead-letter``; its offset is committed in order with the batches around it."""
        self.ms.producer.send(r.topic + BusConsumer.DEAD_LETTER_SUFFIX, r.key, bytes(r.value))
        self.dead_lettered += 1
        self.logger.error("raw batch %s[%d]@%d dead-lettered: %s", r.topic, r.partition, r.offset, err)
        if commit is not None:
            done = _Stepped(None, None, 0, None)
            done.stored = done.published = done.routed = True
            self._submit(done, commit)

    def _on_idle(self):
        self._drain_engine()
        self._raise_store_error()

    def _drain_engine(self):
        """Complete every batch submitted to the engine (overlapped steps)."""
        if self.engine.framed_pending:
            with self._order_lock:
                self._complete(self.engine.drain_framed())

    def _complete(self, done):
        """Results of overlapped steps, in step order: keep what the storage stages need, release the
        record hold and hand the batch to storage."""
        for item, res in done:
            if item.trace is not None:
                item.trace.append(time.perf_counter())
            self.processed_events.mark(res.n_events)
            self._ensure_block(res, item.now)
            hold, item.hold = item.hold, None
            if res.reject_status is not None and len(res.reject_status):
                # per-payload routing runs on a worker thread, in step order; the raw record stays
                # held (readable) until it is done, and the store stage waits for its result
                item.routed_recs = self._router().submit(self._route_and_release, item.batch, res, hold)
            else:
                item.routed_recs = None
                if hold is not None:
                    self._hold(hold, -1)
            item.res, item.batch = res, None
            self._submit(item, item.commit)

    def _router(self):
        pool = self.__dict__.get("_route_pool")
        if pool is None:
            from concurrent.futures import ThreadPoolExecutor
            pool = self._route_pool = ThreadPoolExecutor(1, thread_name_prefix=f"reject-router-{self.tenant.token}")
        return pool

    def _route_and_release(self, batch, res, hold):
        try:
            return self._route(batch, res)
        finally:
            if hold is not None:
                self._hold(hold, -1)

    def _hold(self, at, delta: int):
        """Retention hold (per partition, at its oldest in-flight record) for records the engine
        reads after the consumer's handler returned."""
        t, p, o = at
        with self._hold_lock:
            hs = self._holds.setdefault((t, p), {})
            n = hs.get(o, 0) + delta
            if n > 0:
                hs[o] = n
            else:
                hs.pop(o, None)
            self.ms.instance.bus.hold(t, p, min(hs) if hs else None, holder=self)

    def _raise_store_error(self):
        """A store step failed on the store thread: stop stepping and have the raw consumer re-read
        from the oldest stepped-but-unstored batch of each partition (their results are reused)."""
        if self._store_error is None:
            return
        self.flush()                    # the store thread skips everything queued after the failure
                                        # (batches still in the engine complete first: their results are kept)
        err, self._store_error = self._store_error, None
        rewind: dict = {}
        for (t, p, o) in self._stepped:
            rewind[(t, p)] = min(o, rewind.get((t, p), o))
        raise RetryFrom(rewind, err)

    def process_batch(self, raw: np.ndarray, offs: np.ndarray, now: int | None = None, commit=None, key=None):
        """One synchronous engine step over host arrays (raw payload bytes, u32 offsets); see
        :meth:`process_raw_batch`."""
        with self._order_lock:          # no overlapped submission slips in between the drain and the step
            with self._lock:
                done = self.engine.drain_framed()
            self._complete(done)
            return self.process_raw_batch(RawBatch(len(offs) - 1, int(offs[-1]), raw, offs=offs), now, commit,
                                          key, overlap=False)

    def process_raw_batch(self, batch: RawBatch, now: int | None = None, commit=None, key=None, detach=False,
                          hold=None, overlap: bool | None = None, first: int | None = None):
        """One engine step; storing its rows happens here or, with ``asyncStore``, on the store thread
        while the next step runs (call :meth:`flush` to wait for it).  ``key`` = (topic, partition,
        offset) of the raw record: the result is then kept until stored (see ``_stepped``).
        ``detach``: ``batch`` views memory that is released after this call (a topic record read in
        place), so the bytes the slow path needs are copied.  With overlapped steps the batch is
        only submitted (returns None): it completes when the next batch is submitted or on a drain,
        ``hold`` = (topic, partition, offset) keeps its record retained until then."""
        now = now or now_ms()
        if self.overlap if overlap is None else overlap:
            item = _Stepped(key, None, now, batch, first)
            item.detach, item.commit = detach, commit
            if self.trace is not None:
                item.trace = [time.perf_counter()]
            if key is not None:
                for off in range(item.first, key[2] + 1):
                    self._stepped[(key[0], key[1], off)] = item
            with self._order_lock:
                if hold is not None:
                    item.hold = hold
                    self._hold(hold, +1)
                # not under the tenant lock: the submit waits on the GPU, and the store thread needs
                # that lock to build payloads meanwhile (the engine serialises on its own lock)
                with self.step_timer.time():
                    done = self.engine.submit_framed(batch, now, token=item)
                if item.trace is not None:
                    item.trace.append(time.perf_counter())
                self._complete(done)
            return None
        with self._lock, self.step_timer.time():
            res = self.engine.step_framed(batch, now)
        self.processed_events.mark(res.n_events)
        self._ensure_block(res, now)
        item = _Stepped(key, res, now, None, first)
        item.routed_recs = self._route(batch, res)
        if key is not None:
            for off in range(item.first, key[2] + 1):
                self._stepped[(key[0], key[1], off)] = item
        self._submit(item, commit)
        return res

    def _submit(self, item: "_Stepped", commit):
        if self._store_thread is not None:
            if not item.queued:
                item.queued = True
                self._store_q.put((item, commit))
        else:
            self._store_step(item, commit)

    def _batch_partition(self, bus) -> int:
        """Partition of the next enriched batch.  Unkeyed batches go round-robin, except with
        zero-copy payloads: the topic then holds the engine's pinned row buffers until retention
        drops them, and per-partition retention over round-robin batches would hold partitions x
        the retention window of them -- more than the engine's buffer pool, which then falls back
        to a fresh pinned allocation per step.  Those batches stick to one partition per engine
        (Kafka's sticky partitioner for null keys), so the window is one partition's."""
        if not (self.zero_copy_rows and self.engine_kind == "gpu"):
            return bus.partition_for(self.t_enriched_batches, None)
        if self._sticky_part is None:
            self._sticky_part = bus.partition_for(self.t_enriched_batches, None)
        return self._sticky_part

    def _store_step(self, item: "_Stepped", commit):
        """Storage stages of one stepped batch; each runs once even when the batch is retried."""
        res, now = item.res, item.now
        tr = item.trace
        if tr is not None:
            tr.append(time.perf_counter())
        if not item.stored:
            if self.storage == "durable":
                with self.store_timer.time():
                    if item.payload is None:    # built once: it carries the dictionary deltas
                        item.payload = self.durable_payload(res, item.key, tr)
                    if tr is not None:
                        tr.append(time.perf_counter())
                    n, item.token = self._em().add_durable_batch(item.payload)
                    if tr is not None:
                        tr.append(time.perf_counter())
                self.persisted_events.mark(n)
            elif self.storage == "columnar":
                with self.store_timer.time():
                    if item.payload is None:    # built once: it carries the dictionary deltas
                        item.payload = self.durable_payload(res, item.key, tr) if self.storage == "durable" \
                            else self.columnar_payload(res, now, tr)
                    if tr is not None:
                        tr.append(time.perf_counter())
                    n = self._em().add_columnar_batch(item.payload)
                    if tr is not None:
                        tr.append(time.perf_counter())
                self.persisted_events.mark(n)
            else:
                if item.events is None:
                    item.events = self._to_events(res, now)
                if item.events:
                    self._em().add_enriched_events(item.events)
                    self.persisted_events.mark(len(item.events))
            item.stored = True
        if not item.published:
            with self.publish_timer.time():
                if self.storage in ("columnar", "durable") and self.publish == "batches":
                    bus = self.ms.instance.bus
                    pl = item.payload
                    if self.storage == "durable" and hasattr(bus, "append_arrays") and not isinstance(pl, bytes):
                        # a copy into the log (parallel, GIL released): published in place, the
                        # topic's retention window would hold the engine's pinned block buffers and
                        # grow its pool to that window (measured: slower until it is warm); the
                        # store releases them as soon as they are on disk
                        v = np.asarray(pl).reshape(-1)
                        bus.append_arrays(self.t_enriched_batches, self._batch_partition(bus), np.zeros(1, np.uint8),
                                          np.zeros(2, np.int64), v, np.array([0, v.nbytes], np.int64), ts=now)
                    elif hasattr(bus, "append_external"):   # in place: the log references the payload
                        part = self._batch_partition(bus)
                        if isinstance(pl, bytes):
                            bus.append_bytes(self.t_enriched_batches, part, pl, ts=now)
                        else:
                            bus.append_external(self.t_enriched_batches, part, pl, pl.ctypes.data, pl.nbytes, ts=now)
                    else:
                        self.ms.producer.send(self.t_enriched_batches, None,
                                              pl if isinstance(pl, bytes) else pl.tobytes())
                elif self.publish == "events":
                    self._publish_events(item.events if item.events is not None else self._to_events(res, now))
            item.published = True
        if not item.routed:
            rr = item.routed_recs
            if hasattr(rr, "result"):           # routed on the reject-router thread
                rr = item.routed_recs = rr.result()
            self._send_routed(rr)
            item.routed = True
        if self.storage == "durable" and (self._durable_wait or (item.token or 0) >= 0):
            with self._durable_lock:
                self._durable_wait.append((item, commit))
            if self._store_thread is None:
                self._reap_durable(block=True)
            return
        self._finalize(item, commit)

    def _reap_durable(self, block: bool):
        """Finalize the stored batches whose blocks are durable now (``block``: wait for all)."""
        with self._durable_lock:
            if not self._durable_wait:
                return
            em = self._em()
            try:
                d = em.durable_token()
                while self._durable_wait:
                    item, commit = self._durable_wait[0]
                    if (item.token or 0) > d:
                        if not block:
                            return
                        if not em.wait_durable(item.token, 60.0):
                            raise TimeoutError("event block not durable after 60 s")
                        d = em.durable_token()
                        continue
                    self._durable_wait.popleft()
                    self._finalize(item, commit)
            except Exception:
                # nothing after the failure is durable: those batches are stored again on retry (their
                # enriched batches were published and their rejects routed already: not repeated)
                for item, _ in self._durable_wait:
                    item.stored = False
                    item.token = None
                self._durable_wait.clear()
                raise

    def _finalize(self, item: "_Stepped", commit):
        """A batch is fully stored: it leaves ``_stepped`` and its raw offset commits."""
        tr = item.trace
        if item.key is not None:
            t, p, o = item.key
            for off in range(item.first, o + 1):
                self._stepped.pop((t, p, off), None)
            self._stored_hw[(t, p)] = max(self._stored_hw.get((t, p), -1), o + 1)
        if commit is not None:
            self.ms.instance.bus.commit(self.raw_consumer.group, *commit)
        if tr is not None and self.trace is not None:
            tr.append(time.perf_counter())
            self.trace.append(tr)

    def _store_loop(self):
        while True:
            try:
                # durable blocks in flight: wake up to commit their offsets once they are on disk
                entry = self._store_q.get(timeout=0.002) if self._durable_wait else self._store_q.get()
            except queue.Empty:
                try:
                    self._reap_durable(block=True)
                except Exception as e:  # noqa: BLE001
                    self._store_error = e
                    self.logger.exception("engine store: durable wait failed")
                continue
            try:
                if entry is None:
                    if self._store_error is None:
                        self._reap_durable(block=True)
                    return
                item, commit = entry
                item.queued = False
                if self._store_error is None:   # after a failure nothing is stored (or committed) past it
                    self._store_step(item, commit)
                    self._reap_durable(block=False)
            except Exception as e:  # noqa: BLE001 -- surfaced before the next engine step
                self._store_error = e
                self.logger.exception("engine store step failed")
            finally:
                self._store_q.task_done()

    def flush(self):
        """Complete the batches in the engine, then wait until every queued batch is stored (and its
        raw offset committed) or skipped after a store failure."""
        self._drain_engine()
        if self._store_thread is not None:
            self._store_q.join()
            if self._store_error is None:
                try:
                    self._reap_durable(block=True)          # every stored block on disk, offsets committed
                except Exception as e:  # noqa: BLE001
                    self._store_error = e

    def _dict_deltas(self, tr: list | None = None):
        """(assignment contexts, names) the receiver has not seen yet, and the rule messages."""
        with self._lock:
            if tr is not None:
                tr.append(time.perf_counter())
            asg = {}
            ctx: dict = {}
            for ai in self._asg_dirty:
                a = self._asg_entities.get(ai)
                if a is not None:
                    # event context (reference MongoDeviceEvent) + what enriched-event consumers add
                    # (device token and type, OutboundPayloadEnrichmentLogic.java:54-92)
                    di = self.dev_index.idx.get(a.device_id, -1)
                    asg[ai] = [a.id, a.device_id, a.customer_id, a.area_id, a.asset_id, self._dev_tokens.get(di),
                               self._dev_types.get(di)]
                    # the engine ids the block index trailers key customer / area / asset by
                    for dim, (tok, m) in enumerate(((a.customer_id, self.customers), (a.area_id, self.areas),
                                                    (a.asset_id, self.assets))):
                        if tok is not None and tok in m.idx:
                            ctx.setdefault(dim, {})[tok] = m.idx[tok]
            self._asg_dirty.clear()
            # the engine's host name dictionary grows when a step learns names or rules add alert
            # types (an np.unique over the rows' name ids cost ~10 ms per 1M-row batch)
            if len(self.engine.names) != self._names_known:
                self._names_known = len(self.engine.names)
                self._reload_names()
            names = dict(self._nid2name) if len(self._nid2name) != self._names_sent else {}
            self._names_sent = len(self._nid2name)
        rules = {t.alert_type: t.alert_message for t in self.engine.tests}
        self._ctx_delta = ctx
        return asg, names, rules

    # registries at least this large send their dictionary at start (see _prime_dictionary)
    PRIME_DICTIONARY_MIN = 65536

    def _prime_dictionary(self):
        """Durable storage with a large registry: the assignment contexts go to the event store once,
        at start, before any block (one dictionary record) -- inside the first block's delta, a 1M-
        assignment tenant's first step carried a ~100 MB dictionary and stalled ingest for ~18 s
        (profiles/r6_soak).  Enriched-batch consumers resolve entries they never saw a delta for from
        the store (``EnrichedBatchReader._resolve``)."""
        if self.storage != "durable" or len(self._asg_dirty) < self.PRIME_DICTIONARY_MIN:
            return
        em = self._em()
        if not hasattr(em, "add_durable_dictionary"):
            return
        t0 = time.perf_counter()
        with self._lock:        # no block is encoded between taking the entries and storing them
            asg, names, rules = self._dict_deltas()
            em.add_durable_dictionary(self.block_boot, asg=asg, names=names, rules=rules,
                                      ctx=self._ctx_delta or None)
            self._ctx_delta = None
        self.logger.info("dictionary of %d assignments sent to the event store in %.1f s", len(asg),
                         time.perf_counter() - t0)

    def dictionary_pending(self) -> int:
        """Assignment contexts not yet sent to the event store."""
        return len(self._asg_dirty)

    def durable_payload(self, res, key=None, tr: list | None = None):
        """The step's sealed block + dictionary deltas (``segments.encode_durable_batch``), framed in
        front of the block in its pinned buffer when there is room (no copy; the block then goes to
        the disk with O_DIRECT from that buffer).  ``key`` = (topic, partition, offset) of the raw
        record: the store writes the next offset as the block's commit record, so after a crash the
        tenant resumes exactly behind the last durable block (:meth:`_resume_from_store`)."""
        from ..persistence.segments import encode_durable_batch, frame_durable_batch, set_commit_flag
        asg, names, rules = self._dict_deltas(tr)
        if tr is not None:
            tr.append(time.perf_counter())
        src = None
        if key is not None:
            src = [(self._src_topic(key[0]), key[1], key[2] + 1)]
            set_commit_flag(res.block)
        ctx = getattr(self, "_ctx_delta", None) or None
        if res.block_frame is not None:
            v = frame_durable_batch(res.block_frame, len(res.block), self.boot, asg, names, rules, src, ctx=ctx)
            if v is not None:
                self.zc_framed += 1
                return v
        self.zc_copied += 1
        return encode_durable_batch(res.block, self.boot, asg, names, rules, src, ctx=ctx)

    def _src_topic(self, topic: str) -> str:
        """Input name in commit records: offsets only mean something within one incarnation of the
        bus (a memory-only bus restarts at 0)."""
        return f"{getattr(self.ms.instance.bus, 'incarnation', '')}/{topic}"

    def _resume_from_store(self):
        """Durable storage: move the raw consumer's committed offsets up to what the event store's
        commit records say is on disk (the bus commit trails the disk by one store step, and is lost
        with a volatile bus).  Records behind that offset are never stepped again.  With a checkpoint
        the snapshot owns the offsets instead: the batches after it are replayed to rebuild engine
        state, and the store skips their rows by (boot, sequence)."""
        if self.storage != "durable" or self.ckpt_path:
            return
        bus = self.ms.instance.bus
        em = self._em()
        if not hasattr(em, "durable_source_offset"):
            return
        # store-backed dedup filter: the store may hold no id the filter has forgotten (retention by
        # rows, tightened here), and the filter is seeded with the ids already stored, newest first,
        # so a device re-sending an old payload after a restart is still handed to the store check
        if self.engine.filter_on:
            c = self.engine.cfg
            rows = c.filter_retention_rows(self.filter_retention_slack())
            if hasattr(em, "durable_limit_retention_rows"):
                self.filter_retention_rows = em.durable_limit_retention_rows(rows)
            cap = c.dedup_filter_gens * c.dedup_filter_ids
            count = getattr(em, "durable_alternate_id_count", None)
            self._stored_ids = int(count()) if count is not None else 0
            seeded, skip = 0, 0
            if hasattr(em, "durable_alternate_hashes"):
                self.engine.filter_seed_begin()
                while seeded < cap:
                    h = np.frombuffer(em.durable_alternate_hashes(min(cap - seeded, 1 << 24), skip=skip), np.uint64)
                    if not len(h):
                        break
                    self.engine.filter_seed(h)
                    seeded += len(h)
                    skip += len(h)
            self._stored_ids = max(self._stored_ids, seeded)
            if seeded:
                self.logger.info("dedup filter seeded with %d of %d stored alternate ids", seeded, self._stored_ids)
        group = self.raw_consumer.group
        for topic in self.raw_consumer.topics:
            for p in range(bus.partitions(topic) if hasattr(bus, "partitions") else 1):
                o = em.durable_source_offset(self._src_topic(topic), p)
                if o is not None and o > (bus.committed(group, topic, p) or 0):
                    bus.commit(group, topic, p, o)
                    self.logger.info("resuming %s[%d] at %d (durable in the event store)", topic, p, o)

    def columnar_payload(self, res, now: int, tr: list | None = None) -> bytes:
        """Rows + the dictionary entries the receiver has not seen yet (assignment context, names)."""
        asg, names, rules = self._dict_deltas(tr)
        out = res.out if res.out is not None else np.zeros(0, OUT_REC)
        if tr is not None:
            tr.append(time.perf_counter())
        if self.zero_copy_rows and res.frame_base is not None:
            # header framed in front of the rows in their pinned buffer: no row copy on the host
            v = frame_batch(res.frame_base, out.nbytes, self.boot, res.first_seq, res.world, res.rank, now, asg,
                            names, rules)
            if v is not None:
                self.zc_framed += 1
                return v
        self.zc_copied += 1
        return encode_batch(self.boot, res.first_seq, res.world, res.rank, now, out, asg, names, rules)

    def _publish_events(self, events):
        if events:
            self.ms.producer.send_batch(self.t_enriched, [
                (self._dev_tokens.get(self.dev_index.idx.get(e.device_id, -1)) or e.device_id,
                 payloads.encode_enriched(e, self._context(e))) for e in events])

    def _name(self, nid: int) -> str:
        if nid == NO_NAME:
            return ""
        s = self._nid2name.get(nid)
        if s is None:
            self._reload_names()
            s = self._nid2name.get(nid, "")
        return s

    def _reload_names(self):
        table = self.engine.intern if hasattr(self.engine, "intern") and isinstance(self.engine.intern, dict) \
            else self.engine.intern_table()
        self._nid2name = {i: self.engine.names.get(h, str(h)) for h, i in table.items()}

    def _to_events(self, res, now: int) -> list:
        out = res.out
        if out is None or not len(out):
            return []
        if getattr(res, "block", None) is not None:
            return self._block_events(res)
        eids = res.event_ids()
        tests = self.engine.tests
        events = []
        for r, eid in zip(out, eids):
            a = self._asg_entities.get(int(r["assignment"]))
            if a is None:
                continue
            et = int(r["etype"])
            base = dict(id=f"{self.boot}-{int(eid)}", device_id=a.device_id, device_assignment_id=a.id,
                        customer_id=a.customer_id, area_id=a.area_id, asset_id=a.asset_id,
                        event_date=int(r["event_date"]), received_date=now)
            if et == EV_MEASUREMENT:
                e = DeviceMeasurement(name=self._name(int(r["name_id"])), value=float(r["v0"]), **base)
            elif et == EV_LOCATION:
                e = DeviceLocation(latitude=float(r["v0"]), longitude=float(r["v1"]), **base)
            elif et == EV_ALERT:
                typ = self._name(int(r["name_id"]))
                rule = next((t for t in tests if t.alert_type == typ), None)
                e = DeviceAlert(source=AlertSource.System if rule else AlertSource.Device,
                                level=_LEVELS[min(int(r["level"]), 3)], type=typ,
                                message=rule.alert_message if rule else "", **base)
            elif et == EV_STATE_CHANGE:
                e = DeviceStateChange(attribute="presence", type="presence", previous_state="PRESENT",
                                      new_state="NOT_PRESENT", **base)
            else:
                continue
            events.append(e)
        return events

    def _block_events(self, res) -> list:
        """The step's rows as reference event objects, read from its encoded block: lossless --
        alternate ids, device alert messages, metadata and elevation come back as sent
        (``persistence.segments.materialize_row``, the durable store's own reader)."""
        from ..persistence.segments import decode_block, materialize_row
        blk = res.block
        cols = decode_block(blk if not hasattr(blk, "cpu") else blk.cpu().numpy())
        asg = {}
        for ai in np.unique(cols["asg"]).tolist():
            a = self._asg_entities.get(int(ai))
            if a is not None:
                asg[int(ai)] = [a.id, a.device_id, a.customer_id, a.area_id, a.asset_id]
        names = {int(n): self._name(int(n)) for n in np.unique(cols["name"]).tolist() if int(n) != NO_NAME}
        rules = {t.alert_type: t.alert_message for t in self.engine.tests}
        return [materialize_row(cols, i, asg, names, rules) for i in range(len(cols["etype"]))
                if int(cols["asg"][i]) in asg]

    def _context(self, e) -> dict:
        di = self.dev_index.idx.get(e.device_id, -1)
        return {"deviceId": e.device_id, "deviceToken": self._dev_tokens.get(di),
                "assignmentStatus": "Active", "engine": self.engine_kind}

    # payloads are at least this many bytes on the raw topic (a delimited protobuf request carrying a
    # device token and one event): the most ids a partition's retention can redeliver
    MIN_PAYLOAD_BYTES = 24
    def filter_retention_slack(self) -> int:
        """Rows the store may take beyond its row limit between two retention checks: the blocks in
        flight (steps submitted ahead of the store; the file being written is accounted for by
        ``EngineConfig.filter_retention_rows``)."""
        return 16 * self.engine.cfg.rec_cap

    def check_dedup_sizing(self) -> dict:
        """Runtime check of the engine's dedup sizing (docs/PARITY.md, alternate-id dedup).  The HBM
        window always holds the last ``dedup_slots / 2`` ids.  Without the store-backed filter, a raw
        topic that can redeliver more payloads than that (its retention) lets an old id through
        again.  With it, the filter holds the newest (gens - 1) * ``dedup_filter_ids`` ids and the
        durable store is bounded to that many rows (``_resume_from_store``): warn when the store's
        row limit could not be set that low.  Logs a warning per violated rule; returns the report
        (also ``dedup_sizing_report``)."""
        c = self.engine_cfg
        bus = self.ms.instance.bus
        window = int(c.dedup_slots) // 2
        ids = int(getattr(c, "dedup_filter_ids", 0) or 0)
        redeliver = 0
        for t in self.raw_consumer.topics:
            r = bus.retention(t) if hasattr(bus, "retention") else 0
            parts = bus.partitions(t) if hasattr(bus, "partitions") else 1
            redeliver = -1 if (r <= 0 or redeliver < 0) else redeliver + parts * (r // self.MIN_PAYLOAD_BYTES)
        stored = int(getattr(self, "_stored_ids", 0))
        held = (c.dedup_filter_gens - 1) * ids if ids else 0
        limit = int(getattr(self, "filter_retention_rows", 0) or 0)
        rep = {"window_ids": window, "filter_ids_per_gen": ids, "filter_gens": c.dedup_filter_gens if ids else 0,
               "filter_holds_ids": held, "filter_bytes": c.filter_bytes(),
               "store_retention_rows": limit or None,
               "raw_redeliverable_ids": None if redeliver < 0 else redeliver, "stored_ids": stored,
               "warnings": []}
        if not ids and (redeliver < 0 or redeliver > window):
            rep["warnings"].append(
                f"dedup window holds {window} ids but the raw topic can redeliver "
                f"{'unbounded' if redeliver < 0 else redeliver} payloads and no store-backed filter is "
                f"configured: raise capacity.dedup_slots to >= {2 * max(redeliver, 0) or 'twice the retention'} "
                f"or set capacity.dedup_filter_ids")
        if ids and self.storage == "durable" and (not limit or limit > held):
            rep["warnings"].append(
                f"the durable store keeps {limit or 'unbounded'} rows but the dedup filter holds only the newest "
                f"{held} ids: replays of older stored ids are not caught")
        for w in rep["warnings"]:
            self.logger.warning("%s", w)
        self.dedup_sizing_report = rep
        return rep

    def _watch_filter(self, n_payloads: int, false_pos: int):
        """Filter false positives measured in flight: above 1e-4 of the engine's payloads over a
        window of 2^22, warn (each is a store lookup the step's commit waits for; the generational
        fingerprint filter's rate is ~1e-8 at its sizing load, so this means a probe-bound overflow
        or a mis-sized filter)."""
        w = self._fp_win
        w[0] += false_pos
        w[1] += n_payloads
        if w[1] >= 1 << 22:
            if w[0] > 1e-4 * w[1]:
                self.logger.warning("dedup filter false positives at %.4f%% of payloads (filter %s)",
                                    100.0 * w[0] / w[1], self.engine.filter_state())
                self.dedup_sizing_report.setdefault("warnings", []).append(
                    f"filter false positives {w[0]}/{w[1]}")
            w[0] = w[1] = 0

    def _settle_rechecks(self, res, st):
        """Ids the store-backed filter sent back (SW_ST_RECHECK): one bulk lookup in the durable
        store's alternate-id index.  Ids the store does not hold are the filter's false positives;
        ids whose 64-bit hash it does hold are likely replays, but a hash match is not proof (ADVICE
        r4): both go on to the per-event path, whose alternate-id check compares the id strings
        (``DeviceEventManagement._add``) -- a replay is dropped there, a fresh id that merely
        collides is stored.  The lookup splits the counts: replays vs filter false positives."""
        from ..models.columnar import ST_RECHECK
        rk = st == ST_RECHECK
        n_rk = int(rk.sum())
        n_payloads = int(getattr(res, "n_msgs", 0) or 0)
        if not n_rk:
            self._watch_filter(n_payloads, 0)
            return st
        em = self._em()
        if not hasattr(em, "durable_find_alternate_hashes"):
            return st
        h = np.ascontiguousarray(res.rejects["alt_hash"][rk], np.uint64)
        # indexed blocks only (a binary search each): the raw offsets commit once this step's
        # rejects are routed, so a scan of the blocks the store has not indexed yet would stall the
        # whole pipeline.  An id held only by such a block goes on to the per-event path, whose own
        # store check finds it there: still stored once.
        found = np.frombuffer(em.durable_find_alternate_hashes(h.tobytes(), indexed_only=True), np.uint64)
        n_dup = int(np.isin(h, found).sum()) if len(found) else 0
        self.recheck_duplicates += n_dup
        self.recheck_false_positives += n_rk - n_dup
        self._watch_filter(n_payloads, n_rk - n_dup)
        return st

    def _route(self, batch, res):
        """Route the step's rejected messages like the reference does, per payload: only the payloads
        the reject records point into are parsed (natively, ``pipeline/routing.py``).  Runs while the
        raw record is still readable; the result (the routed records, small) is what the storage
        stage keeps -- never a copy of the batch."""
        from ..pipeline import routing
        st = res.reject_status
        if st is None or not len(st):
            return None
        with self.recheck_timer.time():
            st = self._settle_rechecks(res, st)
        bus = self.ms.instance.bus
        topics = (self.t_unregistered, self.t_registration, self.t_decoded, self.t_failed_decode)
        parts = [bus.partitions(t) if hasattr(bus, "partitions") else 1 for t in topics]
        aux = res.rejects["aux_off"]
        if getattr(batch, "parts", None) is None:
            rr = routing.route_rejects(np.asarray(batch.payload), batch.offsets(), aux, st, "gpu-inbound", parts)
        else:                           # coalesced records: route each record's rejects from its own bytes
            rrs = []
            for part, base in zip(batch.parts, batch.starts):
                m = (aux >= base) & (aux < base + part.payload_bytes)
                if m.any():
                    rrs.append(routing.route_rejects(np.asarray(part.payload), part.offsets(),
                                                     (aux[m] - base).astype(np.uint32), st[m], "gpu-inbound", parts))
            rr = routing.concat(rrs)
        self.routed_payloads += rr.payloads
        return rr

    def _send_routed(self, rr):
        """Publish routed rejects: one native append per (topic, partition) group; acknowledgements /
        streams (rare) are decoded here."""
        from ..pipeline import routing
        if rr is None or not len(rr):
            return
        bus = self.ms.instance.bus
        topics = (self.t_unregistered, self.t_registration, self.t_decoded, self.t_failed_decode)
        prod = self.ms.producer
        for kind, part, kh, ko, vh, vo in rr.groups():
            if kind == routing.CONTROL:
                continue
            if part < 0:                    # no device token (undecodable payload): round-robin
                part = bus.partition_for(topics[kind], None) if hasattr(bus, "partition_for") else 0
            prod.send_arrays(topics[kind], part, kh, ko, vh, vo)
            if kind == routing.UNREGISTERED:
                self.unregistered.mark(len(ko) - 1)
        dec = None
        for _, payload in rr.values(routing.CONTROL):
            dec = dec or ProtobufDecoder()
            try:
                reqs = dec.decode(payload, {})
            except Exception:               # noqa: BLE001 -- the router already parsed it
                continue
            for q in reqs:
                body = {"sourceId": "gpu-inbound", "deviceToken": q["deviceToken"], "originator": q.get("originator"),
                        "eventCreateRequest": {"type": q["type"], "request": q["request"]}}
                prod.send(self.t_decoded, q["deviceToken"], payloads.encode_inbound(body))


class GpuInboundApi:
    def __init__(self, engine: GpuInboundTenantEngine):
        self._e = engine

    def get_statistics(self) -> dict:
        e = self._e
        d = {"processedEvents": e.processed_events.count, "persistedEvents": e.persisted_events.count,
             "unregisteredEvents": e.unregistered.count, "engine": e.engine_kind}
        d.update({f"engine.{k}": v for k, v in e.engine.stats_dict().items()})
        return d

    def get_device_state(self, assignment_id: str) -> dict | None:
        ai = self._e.asg_index.idx.get(assignment_id)
        return None if ai is None else self._e.engine.device_state(ai)

    _INDEX = {"Assignment": 0, "Customer": 2, "Area": 3, "Asset": 4}
    _ETYPE = {"Measurement": EV_MEASUREMENT, "Location": EV_LOCATION, "Alert": EV_ALERT, "StateChange": EV_STATE_CHANGE}

    def list_hot_events(self, event_type: str, index: str, entity_ids: list, start_date: int | None = None,
                        end_date: int | None = None, page_number: int = 1, page_size: int = 100) -> dict:
        """Hot-store read of ``DeviceEventManagement.list*ForIndex`` served from the engine's event ring
        (HBM on the MI355X: one filter kernel over the ring, only the page crosses PCIe).  Events in
        the ring's retention window; older ones live in event management's store."""
        e = self._e
        pos = self._INDEX[index]
        want = set(entity_ids)
        with e._lock:
            asg = [ai for ai, a in e._asg_entities.items()
                   if (a.id, a.device_id, a.customer_id, a.area_id, a.asset_id)[pos] in want]
        total, cols, eids = e.engine.query_store(self._ETYPE[event_type], asg, start_date, end_date, page_number,
                                                 page_size)
        out = []
        rules = {t.alert_type: t.alert_message for t in e.engine.tests}
        for i in range(len(eids)):
            a = e._asg_entities.get(int(cols["asg"][i]))
            if a is None:
                continue
            base = dict(id=f"{e.boot}-{int(eids[i])}", device_id=a.device_id, device_assignment_id=a.id,
                        customer_id=a.customer_id, area_id=a.area_id, asset_id=a.asset_id,
                        event_date=int(cols["date"][i]), received_date=int(cols["recv"][i]))
            et = int(cols["etype"][i])
            name = e.engine.names.get(int(cols["name"][i]), "") if int(cols["name"][i]) else ""
            if et == EV_MEASUREMENT:
                ev = DeviceMeasurement(name=name, value=float(cols["v0"][i]), **base)
            elif et == EV_LOCATION:
                ev = DeviceLocation(latitude=float(cols["v0"][i]), longitude=float(cols["v1"][i]),
                                    elevation=float(cols["v2"][i]), **base)
            elif et == EV_ALERT:
                ev = DeviceAlert(source=AlertSource.System if name in rules else AlertSource.Device,
                                 level=_LEVELS[min(int(cols["level"][i]), 3)], type=name,
                                 message=rules.get(name, ""), **base)
            else:
                ev = DeviceStateChange(attribute="presence", type="presence", previous_state="PRESENT",
                                       new_state="NOT_PRESENT", **base)
            out.append(ev)
        return {"numResults": int(total), "results": out}

    def process_payloads(self, payloads: list) -> dict:
        """Synchronous injection (tests / REST): one engine step over the given wire payloads."""
        raw, offs = pack_messages([bytes(p) for p in payloads])
        r = self._e.process_batch(raw, offs)
        self._e.flush()
        if self._e._store_error is not None:
            err, self._e._store_error = self._e._store_error, None
            raise err
        return {"messages": r.n_msgs, "events": r.n_events, "persisted": r.n_persisted}
