"""service-tenant-management: tenant CRUD, tenant templates, tenant configuration bootstrap (global).

Reference: ``TenantManagementMicroservice.java`` (484), ``TenantTemplateManager.java`` (344),
``TenantBootstrapModelConsumer.java:40-225`` (copy the chosen template into
``/conf/tenants/<id>/`` and write the ``bootstrapped`` marker), ``TenantModelProducer`` (publish
tenant-model updates on ``tenant-model-updates``); RPCs from ``tenant-management.proto`` (8):
CreateTenant, UpdateTenant, GetTenantById, GetTenantByToken, ListTenants, DeleteTenant,
GetTenantTemplates, GetDatasetTemplates.
"""
from __future__ import annotations

import copy
import json
import os
import secrets
import threading

from ..core.errors import ErrorCode, NotFoundException, SiteWhereSystemException
from ..models.domain import SearchCriteria, SearchResults, Tenant, stamp_created, stamp_updated
from ..persistence.store import EntityStore, create_store
from ..runtime.config import dump_document
from ..runtime.microservice import GlobalMicroservice

MULTITENANT_SERVICES = [
    "event-sources", "inbound-processing", "event-management", "device-management", "device-registration",
    "device-state", "rule-processing", "outbound-connectors", "command-delivery", "asset-management",
    "batch-operations", "schedule-management", "label-generation", "streaming-media", "event-search",
]

_MEM = {"datastore": {"type": "memory"}}

# Tenant configuration templates: service identifier -> configuration document.
TENANT_TEMPLATES: dict[str, dict] = {
    "default": {
        "name": "Default (in-memory datastores)",
        "services": {
            "event-sources": {"sources": [{"id": "default-json", "decoder": "json", "receivers": []},
                                          {"id": "default-protobuf", "decoder": "protobuf", "receivers": []}],
                              "deduplicator": {"type": "alternate-id"}},
            "inbound-processing": {"processingThreadCount": 25},
            "event-management": {"datastore": {"type": "memory"}, "buffered": False},
            "device-management": _MEM, "asset-management": _MEM, "batch-operations": _MEM,
            "schedule-management": _MEM, "device-state": _MEM | {"presence": {"checkInterval": "PT10M",
                                                                              "missingInterval": "PT8H"}},
            "device-registration": {"allowNewDevices": True, "defaultDeviceTypeToken": None,
                                    "defaultCustomerToken": None, "defaultAreaToken": None, "autoAssign": True},
            "rule-processing": {"processors": []},
            "outbound-connectors": {"connectors": []},
            "command-delivery": {"router": {"type": "single-choice", "destination": "default"},
                                 "destinations": [{"id": "default", "encoder": "json", "provider": "log"}]},
            "label-generation": {"generators": [{"id": "qrcode", "type": "qrcode"}]},
            "streaming-media": _MEM, "event-search": {"providers": []},
        },
    },
}
TENANT_TEMPLATES["sqlite"] = copy.deepcopy(TENANT_TEMPLATES["default"])
TENANT_TEMPLATES["sqlite"]["name"] = "Durable SQLite datastores"
for _svc in ("device-management", "asset-management", "batch-operations", "schedule-management", "device-state",
             "streaming-media"):
    TENANT_TEMPLATES["sqlite"]["services"][_svc] = {"datastore": {"type": "sqlite",
                                                                  "path": f"/tmp/sitewhere/[[tenant.token]]-{_svc}.db"}}
TENANT_TEMPLATES["sqlite"]["services"]["event-management"] = {
    "datastore": {"type": "sqlite", "path": "/tmp/sitewhere/[[tenant.token]]-events.db"}, "buffered": True}
TENANT_TEMPLATES["cassandra"] = copy.deepcopy(TENANT_TEMPLATES["default"])
TENANT_TEMPLATES["cassandra"]["name"] = "Cassandra event store (time-bucketed partitions)"
# with cassandra.address set (env CASSANDRA_ADDRESS) events go to Cassandra over the native CQL client in the
# reference's table layout; without it the same partition layout is kept in memory (BucketedEventStore)
TENANT_TEMPLATES["cassandra"]["services"]["event-management"] = {
    "datastore": {"type": "cassandra", "address": "${cassandra.address:}", "keyspace": "tenant_[[tenant.token]]",
                  "bucket_ms": 3600000}}
TENANT_TEMPLATES["mongodb"] = copy.deepcopy(TENANT_TEMPLATES["default"])
TENANT_TEMPLATES["mongodb"]["name"] = "MongoDB datastores"
for _svc in ("device-management", "asset-management", "batch-operations", "schedule-management", "device-state",
             "streaming-media"):
    TENANT_TEMPLATES["mongodb"]["services"][_svc] = {"datastore": {"type": "mongodb",
                                                                   "uri": "${mongodb.uri:mongodb://localhost:27017}",
                                                                   "database": "tenant-[[tenant.token]]"}}
# events: the reference's MongoDeviceEventManagement layout with its bulk buffer (200 docs / 250 ms)
TENANT_TEMPLATES["mongodb"]["services"]["event-management"] = {
    "datastore": {"type": "mongodb", "uri": "${mongodb.uri:mongodb://localhost:27017}",
                  "database": "tenant-[[tenant.token]]"}, "buffered": True}
TENANT_TEMPLATES["influxdb"] = copy.deepcopy(TENANT_TEMPLATES["default"])
TENANT_TEMPLATES["influxdb"]["name"] = "InfluxDB event store"
TENANT_TEMPLATES["influxdb"]["services"]["event-management"] = {
    "datastore": {"type": "influxdb", "url": "${influxdb.url:http://localhost:8086}",
                  "database": "tenant-[[tenant.token]]"}, "buffered": True}
# reference templates/stomp: one event source hosting an ActiveMQ-style broker (STOMP transport) and
# decoding JSON batches from its queue
TENANT_TEMPLATES["stomp"] = copy.deepcopy(TENANT_TEMPLATES["default"])
TENANT_TEMPLATES["stomp"]["name"] = "STOMP event source"
TENANT_TEMPLATES["stomp"]["services"]["event-sources"]["sources"] = [
    {"id": "stomp", "decoder": "json-batch",
     "receivers": [{"type": "activemq-broker", "transportUri": "stomp://${stomp.host:127.0.0.1}:${stomp.port:2345}",
                    "queueName": "SITEWHERE.STOMP", "numConsumers": 5}]}]
TENANT_TEMPLATES["gpu"] = copy.deepcopy(TENANT_TEMPLATES["default"])
TENANT_TEMPLATES["gpu"]["name"] = "MI355X-accelerated inbound pipeline"
TENANT_TEMPLATES["gpu"]["services"]["inbound-processing"] = {"engine": "gpu", "batchSize": 65536, "maxDelayMs": 5,
                                                             "storage": "objects", "publishEnriched": "events"}
# protobuf payloads go to the engine undecoded, in micro-batches; JSON keeps the per-event path
TENANT_TEMPLATES["gpu"]["services"]["event-sources"]["sources"][1]["forward"] = "raw"
# JSON device requests reach the engine too, transcoded natively to the protobuf payloads they equal
TENANT_TEMPLATES["gpu"]["services"]["event-sources"]["sources"][0]["forward"] = "raw"
TENANT_TEMPLATES["gpu"]["services"]["event-sources"].update(rawBatchSize=65536, rawMaxDelayMs=5)
# High-throughput MI355X tenant: enriched rows stay columnar end to end (no per-event host objects).
TENANT_TEMPLATES["gpu-columnar"] = copy.deepcopy(TENANT_TEMPLATES["gpu"])
TENANT_TEMPLATES["gpu-columnar"]["name"] = "MI355X pipeline, columnar event store"
# Each engine step's events become one compressed block (~8-16 B/event, encoded on the MI355X) that
# event management appends to durable segment files (O_DIRECT + fdatasync group commit); raw-topic
# offsets are committed once the block is on disk.  Retention by bytes (0 = keep everything).
TENANT_TEMPLATES["gpu-columnar"]["services"]["inbound-processing"].update(
    storage="durable", publishEnriched="batches",
    capacity={"max_msgs": 1 << 18, "max_devices": 65536, "max_assignments": 65536, "store_cap": 1 << 22,
              # alternate-id window: 2^24 slots (512 MB of HBM) hold the last 6-8M ids, so a recheck
              # never scans the blocks the store has not indexed yet
              "dedup_slots": 1 << 24, "gen_cap": 32768,
              # store-backed dedup beyond the window (pipeline/dedup_filter.py): 4 generations of
              # ~2^28 ids (8 GB of the 288 GB of HBM), so the filter holds the newest ~805M ids and
              # forgets older ones; the durable store is bounded to rows the filter still holds
              # (retention by rows, set by the engine at start: ~660M rows, ~12 GB of segments) --
              # every stored id stays checked, false positives ~1e-8, and no cliff as ids accrue.
              "dedup_filter_ids": (1 << 28) - (1 << 21), "dedup_filter_gens": 4})
TENANT_TEMPLATES["gpu-columnar"]["services"]["event-management"] = {
    "datastore": {"type": "segments", "path": "${sitewhere.data.dir:/tmp/sitewhere/data}/[[tenant.token]]/events",
                  "retentionBytes": "${sitewhere.events.retention.bytes:0}"}}
# Per-tenant device cap: gpu-columnar holds 65,536 devices and assignments (its HBM tables and
# the host engine fallback stay small for many tenants per GPU); gpu-columnar-1m is the bench's
# shape -- 1M devices and assignments, 1M-payload steps, state map and window sized for them
# (a few GB of the 288 GB of HBM).  Other sizes: override ``capacity`` in the tenant's
# inbound-processing configuration.
TENANT_TEMPLATES["gpu-columnar-1m"] = copy.deepcopy(TENANT_TEMPLATES["gpu-columnar"])
TENANT_TEMPLATES["gpu-columnar-1m"]["name"] = "MI355X pipeline, columnar event store, 1M devices"
TENANT_TEMPLATES["gpu-columnar-1m"]["services"]["inbound-processing"]["capacity"].update(
    max_msgs=1 << 20, max_devices=(1 << 20) + 65536, max_assignments=(1 << 20) + 65536, store_cap=1 << 23,
    gen_cap=1 << 19, state_slots=1 << 24, dedup_filter_ids=(1 << 29) - (1 << 22))
# a million devices and assignments live in the process: keep them out of the cyclic GC (a full
# collection over them paused ingest for seconds every ~45 s, profiles/r6_soak)
TENANT_TEMPLATES["gpu-columnar-1m"]["services"]["inbound-processing"]["tuneGc"] = True
TENANT_TEMPLATES["gpu-columnar-1m"]["services"]["event-sources"].update(rawBatchSize=1 << 20)
# volatile variant (benchmarks of the pipeline alone): rows kept in host memory, newest 2^28 held
TENANT_TEMPLATES["gpu-memory"] = copy.deepcopy(TENANT_TEMPLATES["gpu-columnar"])
TENANT_TEMPLATES["gpu-memory"]["name"] = "MI355X pipeline, in-memory columnar event store"
TENANT_TEMPLATES["gpu-memory"]["services"]["inbound-processing"]["storage"] = "columnar"
TENANT_TEMPLATES["gpu-memory"]["services"]["event-management"] = {"datastore": {"type": "columnar",
                                                                                "retentionRows": 1 << 28}}

class TenantManagement:
    TENANTS = "tenants"

    def __init__(self, store: EntityStore | None = None, on_change=None):
        self._s = store or create_store("memory")
        self._s.register(self.TENANTS, Tenant, ("token",))
        self._on_change = on_change or (lambda kind, t: None)

    def create_tenant(self, request: dict) -> Tenant:
        token = request.get("token")
        if not token:
            raise SiteWhereSystemException(ErrorCode.IncompleteData, detail="tenant token required")
        if self._s.get_by_token(self.TENANTS, token):
            raise SiteWhereSystemException(ErrorCode.DuplicateTenantToken, detail=token)
        tpl = request.get("configurationTemplateId", "default")
        if tpl not in TENANT_TEMPLATES:
            raise SiteWhereSystemException(ErrorCode.InvalidTemplate, detail=tpl)
        t = Tenant(token=token, name=request.get("name", token),
                   authentication_token=request.get("authenticationToken") or secrets.token_hex(12),
                   authorized_user_ids=list(request.get("authorizedUserIds", [])),
                   configuration_template_id=tpl,
                   dataset_template_id=request.get("datasetTemplateId", "empty"),
                   image_url=request.get("imageUrl"), metadata=dict(request.get("metadata", {})))
        stamp_created(t)
        t = self._s.put(self.TENANTS, t)
        self._on_change("created", t)
        return t

    def update_tenant(self, id: str, request: dict) -> Tenant:
        t = self._require_id(id)
        for k, f in (("name", "name"), ("authenticationToken", "authentication_token"), ("imageUrl", "image_url"),
                     ("authorizedUserIds", "authorized_user_ids"), ("metadata", "metadata")):
            if k in request:
                setattr(t, f, request[k])
        stamp_updated(t)
        t = self._s.put(self.TENANTS, t)
        self._on_change("updated", t)
        return t

    def get_tenant(self, id: str) -> Tenant | None:
        return self._s.get(self.TENANTS, id)

    get_tenant_by_id = get_tenant

    def get_tenant_by_token(self, token: str) -> Tenant | None:
        return self._s.get_by_token(self.TENANTS, token)

    def list_tenants(self, criteria: SearchCriteria | None = None, text_search: str | None = None,
                     user_id: str | None = None) -> SearchResults:
        c = criteria or SearchCriteria(page_size=0)

        def pred(t: Tenant):
            if text_search and text_search.lower() not in (t.name + t.token).lower():
                return False
            if user_id and user_id not in t.authorized_user_ids:
                return False
            return True

        ts = self._s.query(self.TENANTS, pred, sort_key=lambda t: t.name)
        return SearchResults(len(ts), c.slice(ts))

    def delete_tenant(self, id: str) -> Tenant:
        t = self._require_id(id)
        self._s.delete(self.TENANTS, id)
        self._on_change("deleted", t)
        return t

    def get_tenant_templates(self) -> list[dict]:
        return [{"id": k, "name": v["name"]} for k, v in sorted(TENANT_TEMPLATES.items())]

    def get_dataset_templates(self) -> list[dict]:
        from .dataset_runner import dataset_templates
        return [{k: v for k, v in meta.items() if k != "initializers"} for _, meta in
                sorted(dataset_templates().items())]

    def _require_id(self, id: str) -> Tenant:
        t = self._s.get(self.TENANTS, id)
        if t is None:
            raise NotFoundException(ErrorCode.InvalidTenantToken, id)
        return t


class TenantManagementMicroservice(GlobalMicroservice):
    identifier = "tenant-management"
    name = "Tenant Management"

    def __init__(self, instance, hostname=None, store: EntityStore | None = None):
        super().__init__(instance, hostname)
        self._store = store
        self.tenants: TenantManagement | None = None
        self._lock = threading.Lock()
        # a reference deployment's Spring XML tenant templates, imported as ref-<name>
        ref = os.environ.get("SITEWHERE_REFERENCE_TEMPLATES")
        if ref:
            from ..runtime.xml_import import register_reference_templates
            register_reference_templates(ref)

    def default_configuration(self) -> dict:
        return {"datastore": {"type": "memory"}}

    def register_services(self, resolver):
        self.tenants = TenantManagement(self._store, on_change=self._tenant_changed)
        resolver.add_global("TenantManagement", self.tenants)

    # TenantModelProducer + TenantBootstrapModelConsumer, fused: publish the model update and
    # (idempotently) copy the template into the tenant's configuration subtree.
    def _tenant_changed(self, kind: str, t: Tenant):
        inst = self.instance
        self.producer.send(inst.naming.tenant_model_updates(), t.token,
                           json.dumps({"type": kind, "tenant": t.to_dict()}).encode())
        if kind == "created":
            self.bootstrap_tenant_configuration(t)
        elif kind == "deleted":
            try:
                inst.coord.delete(inst.tenant_conf_path(t.token), recursive=True)
            except KeyError:
                pass

    def bootstrap_tenant_configuration(self, t: Tenant):
        inst = self.instance
        with self._lock:
            if inst.coord.exists(inst.tenant_conf_path(t.token, "bootstrapped")):
                return
            tpl = TENANT_TEMPLATES[t.configuration_template_id]
            for svc, doc in tpl["services"].items():
                inst.coord.put(inst.tenant_conf_path(t.token, f"{svc}.json"), dump_document(doc))
            inst.coord.ensure(inst.tenant_conf_path(t.token, "bootstrapped"))

    def configuration_updated(self, doc):
        pass


def bootstrap_default_tenant(tm: TenantManagement):
    """Instance template initializer (reference tenantModel.groovy)."""
    if tm.get_tenant_by_token("default") is None:
        tm.create_tenant({"token": "default", "name": "Default Tenant", "authenticationToken": "sitewhere1234567890",
                          "authorizedUserIds": ["admin", "noadmin"], "configurationTemplateId": "default",
                          "datasetTemplateId": "construction"})
