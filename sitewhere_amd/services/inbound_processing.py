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


class InboundProcessingTenantEngine(MicroserviceTenantEngine):
    def tenant_initialize(self, monitor):
        ms, t = self.ms, self.tenant.token
        n = ms.instance.naming
        self.t_unregistered = n.unregistered_device_events(t)
        self.t_enriched = n.inbound_enriched_events(t)
        self.t_enriched_cmd = n.enriched_command_invocations(t)
        self.devices = NearCache(5000, 60.0)
        self.assignments = NearCache(5000, 60.0)
        # processingThreadCount (reference default 25) is honoured, capped by what helps here:
        # Python threads contend on the GIL, so work runs batched on few threads and the bulk
        # throughput path is the fused GPU engine (``"engine": "gpu"``).
        threads = int(self.config.get("processingThreadCount", 25))
        self.decoded_consumer = BusConsumer(self, "decoded-event-consumers", [n.decoded_events(t), n.inbound_reprocess_events(t)],
                                            self._process_decoded, threads=min(threads, int(self.config.get("maxThreads", 2))))
        self.persisted_consumer = BusConsumer(self, "persisted-event-consumers", [n.inbound_persisted_events(t)],
                                              self._process_persisted, threads=min(10, int(self.config.get("maxThreads", 2))))
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
        for r in recs:
            m = json.loads(r.value)
            e = codec.from_wire(m["entity"])
            if m["kind"].startswith("device."):
                self.devices.invalidate(getattr(e, "token", None))
                self.devices.invalidate(("id", e.id))
            elif m["kind"].startswith("assignment."):
                self.assignments.invalidate(e.id)
                self.devices.invalidate(("id", e.device_id))
                self.devices.invalidate(None)

    def device_by_token(self, token):
        with self.device_lookup.time():
            return self.devices.get(token, lambda k: self._dm().get_device_by_token(k))

    def assignment(self, aid):
        with self.assignment_lookup.time():
            return self.assignments.get(aid, lambda k: self._dm().get_device_assignment(k))

    # ---- InboundPayloadProcessingLogic -----------------------------------------------
    def _process_decoded(self, recs):
        """Validate a poll batch, then store it with one event-management call per (assignment, type)
        run -- the reference issues one async gRPC per event (UnaryEventStorageStrategy); batching
        keeps per-key order (records of one device are in one partition, in order)."""
        em = self._em()
        groups: dict = {}
        order: list = []
        for r in recs:
            try:
                p = payloads.decode_inbound(r.value)
                a = self._validate(p)
                if a is None:
                    continue
                req = p["eventCreateRequest"]
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
        for key in order:
            reqs = groups[key]
            # A storage failure is transient (event management unavailable / restarting): retry the
            # call in place, then fail the batch so the consumer re-reads it from its first record
            # (at-least-once; alternate-id idempotent storage absorbs the replayed prefix).  Only
            # malformed payloads (above) are counted as failed and skipped.
            for attempt in range(4):
                try:
                    with self.event_storage.time():
                        getattr(em, key[1])(key[0], reqs)
                    self.processed_events.mark(len(reqs))
                    break
                except Exception:
                    if attempt == 3:
                        self.logger.warning("storing %d events failed; batch will be redelivered", len(reqs))
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
        out, cmds = [], []
        for r in recs:
            ev = payloads.decode_persisted(r.value)
            a = self.assignment(ev.device_assignment_id)
            if a is None:
                continue
            dev = self.devices.get(("id", a.device_id), lambda k: self._dm().get_device(k[1]))
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
