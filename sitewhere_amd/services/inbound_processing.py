"""service-inbound-processing: validate decoded events, persist them, enrich persisted events.

Reference: ``service-inbound-processing`` --
  * ``DecodedEventsConsumer.java:79-204`` subscribes to decoded + reprocess topics and runs
    ``InboundPayloadProcessingLogic.java:101-218`` per record: device lookup by token, then the
    active assignment; unregistered/unassigned devices go to the unregistered topic; otherwise
    ``UnaryEventStorageStrategy.java:53-90`` calls event-management ``add*`` by event type.
    (The reference runs this on the poll thread although 25 threads are configured; here
    ``processingThreadCount`` is honoured.)
  * ``PersistedEventsConsumer.java:50-142`` (10 threads) + ``OutboundPayloadEnrichmentLogic.java:54-92``:
    attach device + assignment context, send to the enriched topic keyed by device token, and
    command invocations additionally to the enriched-command-invocations topic.
  * ``CachedDeviceManagementApiChannel`` + near cache for the lookups.
The MI355X mode (``"engine": "gpu"``) replaces both consumers with :class:`GpuInboundEngine` over raw
payload batches (see :mod:`sitewhere_amd.services.gpu_inbound`).
"""
from __future__ import annotations

import json
import time

from ..models.domain import DeviceAssignmentStatus, DeviceEventType
from ..rpc import codec
from ..runtime.consumers import BusConsumer, NearCache
from ..runtime.microservice import MicroserviceTenantEngine, MultitenantMicroservice
from ..bus import payloads

_ADDERS = {
    "DeviceMeasurement": "add_measurements", "DeviceLocation": "add_locations", "DeviceAlert": "add_alerts",
    "DeviceCommandResponse": "add_command_responses", "Acknowledge": "add_command_responses",
    "DeviceStateChange": "add_state_changes", "DeviceCommandInvocation": "add_command_invocations",
}
# request type -> event type of event management's batch add (``add_event_batch``); command
# invocations keep their per-assignment add (their target defaults to the assignment)
_BATCH_TYPES = {"DeviceMeasurement": "Measurement", "DeviceLocation": "Location", "DeviceAlert": "Alert",
                "DeviceCommandResponse": "CommandResponse", "Acknowledge": "CommandResponse",
                "DeviceStateChange": "StateChange"}


def model_changes(recs) -> list:
    """(kind, entity) of the device-model change feed's records, in order; bulk records (a bulk
    create's entities, ``DeviceManagementTenantEngine._publish_changes``) expanded."""
    out = []
    for r in recs:
        m = json.loads(r.value)
        if m["kind"] == "bulk":
            kind = m["of"]
            out.extend((kind, codec.from_wire(w)) for w in m["entities"])
        else:
            out.append((m["kind"], codec.from_wire(m["entity"])))
    return out


class InboundProcessingTenantEngine(MicroserviceTenantEngine):
    def tenant_initialize(self, monitor):
        ms, t = self.ms, self.tenant.token
        n = ms.instance.naming
        self.t_unregistered = n.unregistered_device_events(t)
        self.t_enriched = n.inbound_enriched_events(t)
        self.t_enriched_cmd = n.enriched_command_invocations(t)
        self.devices = NearCache(5000, 60.0)
        self.assignments = NearCache(5000, 60.0)
        self._dev_token: dict = {}              # device id -> token, for cache invalidation by id
        # processingThreadCount (reference default 25) is honoured, capped by what helps here:
        # Python threads contend on the GIL, so work runs batched on few threads and the bulk
        # throughput path is the fused GPU engine (``"engine": "gpu"``).
        threads = int(self.config.get("processingThreadCount", 25))
        # a poll of up to 4096 records across partitions per handler call: one bulk device lookup and
        # one event-management batch per poll (DecodedEventsConsumer.java:155-204 batches per poll too)
        self.decoded_consumer = BusConsumer(self, "decoded-event-consumers", [n.decoded_events(t), n.inbound_reprocess_events(t)],
                                            self._process_decoded, threads=min(threads, int(self.config.get("maxThreads", 2))),
                                            max_records=4096, merge_partitions=True)
        self.persisted_consumer = BusConsumer(self, "persisted-event-consumers", [n.inbound_persisted_events(t)],
                                              self._process_persisted, threads=min(10, int(self.config.get("maxThreads", 2))),
                                              max_records=4096, merge_partitions=True)
        self.processed_events = self.create_meter("processedEvents")
        self.failed_events = self.create_meter("failedEvents")
        self.device_lookup = self.create_timer("deviceLookup")
        self.assignment_lookup = self.create_timer("assignmentLookup")
        self.event_storage = self.create_timer("eventStorage")
        self.unregistered = self.create_meter("unregisteredEvents")
        # invalidate near caches from the device-model change feed; a control-plane consumer: an
        # update that keeps failing is retried (and alerted on), never dead-lettered and skipped
        self.model_consumer = BusConsumer(self, "model-updates", [n.tenant_prefix(t) + "device-model-updates"],
                                          self._on_model_update, max_attempts=None)
        self.api = {"InboundProcessing": InboundProcessingApi(self)}

    def tenant_start(self, monitor):
        for c in (self.model_consumer, self.decoded_consumer, self.persisted_consumer):
            self.start_nested_component(c, monitor, require=True)

    def tenant_stop(self, monitor):
        for c in (self.decoded_consumer, self.persisted_consumer, self.model_consumer):
            c.lifecycle_stop(monitor)

    def _dm(self):
        return self.ms.api("DeviceManagement", self.tenant.token)

    def _em(self):
        return self.ms.api("DeviceEventManagement", self.tenant.token)

    def _on_model_update(self, recs):
        self._apply_model_changes(model_changes(recs))

    def _apply_model_changes(self, changes):
        for kind, e in changes:
            if kind.startswith("device."):
                self.devices.invalidate(getattr(e, "token", None))
                self.devices.invalidate(("id", e.id))
            elif kind.startswith("assignment."):
                # the device's cached entries carry its assignment id: drop them (by id, and by the
                # token it was loaded under)
                self.assignments.invalidate(e.id)
                self.devices.invalidate(("id", e.device_id))
                tok = self._dev_token.get(e.device_id)
                if tok is not None:
                    self.devices.invalidate(tok)

    def device_by_token(self, token):
        with self.device_lookup.time():
            d = self.devices.get(token, lambda k: self._dm().get_device_by_token(k))
        if d is not None:
            self._dev_token[d.id] = token
        return d

    def _load_devices(self, tokens):
        dm = self._dm()
        if hasattr(dm, "get_devices_by_tokens"):
            return dm.get_devices_by_tokens(list(tokens))
        return [dm.get_device_by_token(t) for t in tokens]

    def _load_assignments(self, ids):
        dm = self._dm()
        if hasattr(dm, "get_device_assignments"):
            return dm.get_device_assignments(list(ids))
        return [dm.get_device_assignment(i) for i in ids]

    def _load_devices_by_id(self, keys):
        dm = self._dm()
        ids = [k[1] for k in keys]
        if hasattr(dm, "get_devices"):
            return dm.get_devices(ids)
        return [dm.get_device(i) for i in ids]

    def assignment(self, aid):
        with self.assignment_lookup.time():
            return self.assignments.get(aid, lambda k: self._dm().get_device_assignment(k))

    # ---- InboundPayloadProcessingLogic -----------------------------------------------
    def _process_decoded(self, recs):
        """Validate a whole poll batch in one pass -- the near cache answers what it holds and every
        miss (devices by token, then their assignments) is fetched with ONE bulk lookup -- then store
        it with ONE event-management call (``add_event_batch``; per-key order kept: a device's
        records are in one partition, in order).  The reference validates and stores per event on
        the poll thread (DecodedEventsConsumer.java:155-204, UnaryEventStorageStrategy.java:53-90)
        and batches only inside the Mongo buffer (DeviceEventBuffer.java:99-135).  Command
        invocations keep one call per (assignment) run."""
        em = self._em()
        decoded = []
        for r in recs:
            try:
                decoded.append(payloads.decode_inbound(r.value))
            except Exception:
                self.failed_events.mark()
                self.logger.exception("failed to decode inbound payload")
        with self.device_lookup.time():
            devs = self.devices.get_many([p["deviceToken"] for p in decoded], self._load_devices)
        for tok, d in devs.items():
            if d is not None:
                self._dev_token[d.id] = tok
        with self.assignment_lookup.time():
            asgs = self.assignments.get_many([d.device_assignment_id for d in devs.values()
                                              if d is not None and d.device_assignment_id], self._load_assignments)
        items, groups, order = [], {}, []
        for p in decoded:
            try:
                d = devs.get(p["deviceToken"])
                a = asgs.get(d.device_assignment_id) if d is not None and d.device_assignment_id else None
                if d is None or a is None or a.status == DeviceAssignmentStatus.Released:
                    self.unregistered.mark()
                    self.ms.producer.send(self.t_unregistered, p["deviceToken"], payloads.encode_inbound(p))
                    continue
                req = p["eventCreateRequest"]
                et = _BATCH_TYPES.get(req["type"])
                if et is not None and hasattr(em, "add_event_batch"):
                    items.append((a.id, et, req["request"]))
                    continue
                fn = _ADDERS.get(req["type"])
                if fn is None:
                    self._route_stream(p, a)
                    continue
                key = (a.id, fn)
                if key not in groups:
                    groups[key] = []
                    order.append(key)
                groups[key].append(req["request"])
            except Exception:
                self.failed_events.mark()
                self.logger.exception("failed to process inbound payload")
        calls = [(lambda: em.add_event_batch(items), len(items))] if items else []
        calls += [(lambda key=key: getattr(em, key[1])(key[0], groups[key]), len(groups[key])) for key in order]
        for call, n in calls:
            # A storage failure is transient (event management unavailable / restarting): retry the
            # call in place, then fail the batch so the consumer re-reads it from its first record
            # (at-least-once; alternate-id idempotent storage absorbs the replayed prefix).  Only
            # malformed payloads (above) are counted as failed and skipped.
            for attempt in range(4):
                try:
                    with self.event_storage.time():
                        call()
                    self.processed_events.mark(n)
                    break
                except Exception:
                    if attempt == 3:
                        self.logger.warning("storing %d events failed; batch will be redelivered", n)
                        raise
                    time.sleep(0.02 * (1 << attempt))

    def _validate(self, p: dict):
        token = p["deviceToken"]
        device = self.device_by_token(token)
        a = None
        if device is not None and device.device_assignment_id:
            a = self.assignment(device.device_assignment_id)
        if device is None or a is None or a.status == DeviceAssignmentStatus.Released:
            self.unregistered.mark()
            self.ms.producer.send(self.t_unregistered, token, payloads.encode_inbound(p))
            return None
        return a

    def _route_stream(self, p: dict, a):
        """Device stream requests go to streaming media (reference IInboundEventProcessor
        onDeviceStreamCreateRequest / onDeviceStreamDataCreateRequest)."""
        req = p["eventCreateRequest"]
        t = req["type"]
        if t not in ("DeviceStream", "DeviceStreamData", "SendDeviceStreamData"):
            return
        sm = self.ms.api("StreamingMedia", self.tenant.token)
        r = req["request"]
        if t == "DeviceStream":
            ack = sm.handle_device_stream_request(p["deviceToken"], r)
            self._system_command(p["deviceToken"], {"type": "DeviceStreamAck", **ack})
        elif t == "SendDeviceStreamData":
            # device asks for a chunk: answer with a system command carrying the stored bytes
            chunk = sm.get_device_stream_data(a.id, r["streamId"], int(r.get("sequenceNumber", 0)))
            self._system_command(p["deviceToken"], {
                "type": "DeviceStreamData", "streamId": r["streamId"],
                "sequenceNumber": int(r.get("sequenceNumber", 0)),
                "data": chunk.data if chunk is not None else b""})
        else:
            data = r.get("data") or b""
            sm.add_device_stream_data(a.id, r["streamId"], int(r.get("sequenceNumber", 0)),
                                      data if isinstance(data, bytes) else bytes(data), r.get("eventDate"))

    def _system_command(self, device_token: str, command: dict):
        try:
            self.ms.api("CommandDelivery", self.tenant.token, wait_s=1.0).deliver_system_command(device_token, command)
        except Exception:
            self.logger.warning("system command %s to %s not delivered", command.get("type"), device_token)

    def process_payload(self, p: dict, em=None):
        a = self._validate(p)
        if a is None:
            return None
        req = p["eventCreateRequest"]
        fn = _ADDERS.get(req["type"])
        if fn is None:
            return None
        with self.event_storage.time():
            return getattr(em or self._em(), fn)(a.id, req["request"])

    # ---- OutboundPayloadEnrichmentLogic -------------------------------------------
    def _process_persisted(self, recs):
        """Enrich a poll batch of persisted events (OutboundPayloadEnrichmentLogic.java:54-92): the
        batch's assignments and devices come from the near cache, misses in one bulk lookup each."""
        out, cmds = [], []
        evs = [payloads.decode_persisted(r.value) for r in recs]
        with self.assignment_lookup.time():
            asgs = self.assignments.get_many([ev.device_assignment_id for ev in evs], self._load_assignments)
        with self.device_lookup.time():
            devs = self.devices.get_many([("id", a.device_id) for a in asgs.values() if a is not None],
                                         self._load_devices_by_id)
        for ev in evs:
            a = asgs.get(ev.device_assignment_id)
            if a is None:
                continue
            dev = devs.get(("id", a.device_id))
            ctx = {"deviceId": a.device_id, "deviceToken": dev.token if dev else None,
                   "deviceTypeId": a.device_type_id, "parentDeviceId": dev.parent_device_id if dev else None,
                   "deviceStatus": dev.status if dev else None, "deviceMetadata": dev.metadata if dev else {},
                   "assignmentStatus": a.status.value, "assignmentMetadata": a.metadata}
            body = payloads.encode_enriched(ev, ctx)
            key = ctx["deviceToken"] or a.device_id
            out.append((key, body))
            if ev.event_type == DeviceEventType.CommandInvocation:
                cmds.append((key, body))
        if out:
            self.ms.producer.send_batch(self.t_enriched, out)
        if cmds:
            self.ms.producer.send_batch(self.t_enriched_cmd, cmds)


class InboundProcessingApi:
    def __init__(self, engine):
        self._e = engine

    def get_statistics(self) -> dict:
        e = self._e
        return {"processedEvents": e.processed_events.count, "failedEvents": e.failed_events.count,
                "unregisteredEvents": e.unregistered.count, "deviceCacheHits": e.devices.hits,
                "deviceCacheMisses": e.devices.misses}


class InboundProcessingMicroservice(MultitenantMicroservice):
    identifier = "inbound-processing"
    name = "Inbound Processing"

    def service_names(self):
        return ["InboundProcessing"]

    def create_tenant_engine(self, tenant):
        cfg = self.tenant_configuration(tenant.token)
        if cfg.get("engine") == "gpu":
            from .gpu_inbound import GpuInboundTenantEngine
            return GpuInboundTenantEngine(self, tenant)
        return InboundProcessingTenantEngine(self, tenant)
