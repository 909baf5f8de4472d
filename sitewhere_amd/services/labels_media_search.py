"""service-label-generation, service-streaming-media and service-event-search (multitenant).

* label generation -- ``QrCodeGenerator.java:37-70``; RPCs (``label-generation.proto``, 10):
  Get{CustomerType,Customer,AreaType,Area,DeviceType,Device,DeviceGroup,DeviceAssignment,AssetType,Asset}Label
* streaming media -- ``DeviceStreamManager.java:36``: stream creation acks and chunked stream data
  (sequence numbers), data requests answered from storage
* event search -- ``SearchProviderManager`` + ``SolrSearchProvider.java:51``: external search providers
  (Solr over HTTP) and an in-process provider over the tenant's event store
"""
from __future__ import annotations

import json
import urllib.parse
import urllib.request

from ..core.errors import ErrorCode, NotFoundException, SiteWhereSystemException
from ..models.domain import DeviceStreamData, Label, SearchResults, now_ms
from ..persistence.store import create_store
from ..runtime.microservice import MicroserviceTenantEngine, MultitenantMicroservice
from .qrcode import QrCode


# ============================================================================ labels
class LabelGeneration:
    ENTITIES = {
        "customer_type": ("DeviceManagement", "get_customer_type", "customertype"),
        "customer": ("DeviceManagement", "get_customer", "customer"),
        "area_type": ("DeviceManagement", "get_area_type", "areatype"),
        "area": ("DeviceManagement", "get_area", "area"),
        "device_type": ("DeviceManagement", "get_device_type", "devicetype"),
        "device": ("DeviceManagement", "get_device", "device"),
        "device_group": ("DeviceManagement", "get_device_group", "devicegroup"),
        "device_assignment": ("DeviceManagement", "get_device_assignment", "assignment"),
        "asset_type": ("AssetManagement", "get_asset_type", "assettype"),
        "asset": ("AssetManagement", "get_asset", "asset"),
    }

    def __init__(self, engine, generators: dict):
        self._e = engine
        self._gens = generators

    def _label(self, kind: str, generator_id: str, entity_id: str) -> Label:
        g = self._gens.get(generator_id)
        if g is None:
            raise NotFoundException(ErrorCode.Error, f"label generator {generator_id}")
        svc, getter, path = self.ENTITIES[kind]
        ent = getattr(self._e.ms.api(svc, self._e.tenant.token), getter)(entity_id)
        if ent is None:
            raise NotFoundException(ErrorCode.Error, f"{kind} {entity_id}")
        url = g.get("baseUrl", "sitewhere://{tenant}/{path}/{token}").format(
            tenant=self._e.tenant.token, path=path, token=getattr(ent, "token", None) or ent.id)
        qr = QrCode(url, ec=g.get("ecLevel", "M"))
        return Label("image/png", qr.to_png(int(g.get("scale", 6))))

    def get_customer_type_label(self, g, i): return self._label("customer_type", g, i)
    def get_customer_label(self, g, i): return self._label("customer", g, i)
    def get_area_type_label(self, g, i): return self._label("area_type", g, i)
    def get_area_label(self, g, i): return self._label("area", g, i)
    def get_device_type_label(self, g, i): return self._label("device_type", g, i)
    def get_device_label(self, g, i): return self._label("device", g, i)
    def get_device_group_label(self, g, i): return self._label("device_group", g, i)
    def get_device_assignment_label(self, g, i): return self._label("device_assignment", g, i)
    def get_asset_type_label(self, g, i): return self._label("asset_type", g, i)
    def get_asset_label(self, g, i): return self._label("asset", g, i)

    def list_label_generators(self) -> list[dict]:
        return [{"id": k, **v} for k, v in self._gens.items()]


class LabelGenerationTenantEngine(MicroserviceTenantEngine):
    def tenant_initialize(self, monitor):
        gens = {g["id"]: g for g in self.config.get("generators", [{"id": "qrcode", "type": "qrcode"}])}
        self.api = {"LabelGeneration": LabelGeneration(self, gens)}


class LabelGenerationMicroservice(MultitenantMicroservice):
    identifier = "label-generation"
    name = "Label Generation"

    def service_names(self):
        return ["LabelGeneration"]

    def create_tenant_engine(self, tenant):
        return LabelGenerationTenantEngine(self, tenant)


# ============================================================================ streaming media
class DeviceStreamManager:
    """Stream data chunks per (assignment, stream), reassembled in sequence order
    (``DeviceStreamManager.java``).  Chunks live in the tenant's configured datastore (memory, SQLite,
    MongoDB...; the reference's Mongo / Cassandra stream stores throw "not supported"), keyed by
    (assignment, stream, sequence number) so a re-sent chunk replaces itself."""

    COLLECTION = "deviceStreamData"

    def __init__(self, engine, store=None):
        self._e = engine
        self._store = store or create_store("memory")
        self._store.register(self.COLLECTION, DeviceStreamData, ())

    def _dm(self):
        return self._e.ms.api("DeviceManagement", self._e.tenant.token)

    def handle_device_stream_request(self, device_token: str, request: dict) -> dict:
        dm = self._dm()
        dev = dm.get_device_by_token(device_token)
        if dev is None or not dev.device_assignment_id:
            return {"streamId": request.get("streamId"), "state": "STREAM_FAILED"}
        if dm.get_device_stream_by_stream_id(dev.device_assignment_id, request["streamId"]):
            return {"streamId": request["streamId"], "state": "STREAM_EXISTS"}
        dm.create_device_stream(dev.device_assignment_id, {"streamId": request["streamId"],
                                                           "contentType": request.get("contentType", ""),
                                                           "metadata": request.get("metadata", {})})
        return {"streamId": request["streamId"], "state": "STREAM_CREATED"}

    @staticmethod
    def _key(assignment_id: str, stream_id: str, seq: int) -> str:
        return f"{assignment_id}:{stream_id}:{int(seq)}"

    def add_device_stream_data(self, assignment_id: str, stream_id: str, sequence_number: int, data: bytes,
                               event_date: int | None = None) -> DeviceStreamData:
        if self._dm().get_device_stream_by_stream_id(assignment_id, stream_id) is None:
            raise SiteWhereSystemException(ErrorCode.InvalidStreamId, detail=stream_id)
        d = DeviceStreamData(id=self._key(assignment_id, stream_id, sequence_number),
                             device_assignment_id=assignment_id, stream_id=stream_id,
                             sequence_number=int(sequence_number), data=bytes(data),
                             event_date=event_date or now_ms(), received_date=now_ms())
        return self._store.put(self.COLLECTION, d)

    def get_device_stream_data(self, assignment_id: str, stream_id: str, sequence_number: int):
        return self._store.get(self.COLLECTION, self._key(assignment_id, stream_id, sequence_number))

    def list_device_stream_data(self, assignment_id: str, stream_id: str) -> SearchResults:
        chunks = self._store.query(self.COLLECTION, lambda d: d.device_assignment_id == assignment_id and
                                   d.stream_id == stream_id, sort_key=lambda d: d.sequence_number)
        return SearchResults(len(chunks), chunks)

    def get_stream_content(self, assignment_id: str, stream_id: str) -> bytes:
        return b"".join(d.data for d in self.list_device_stream_data(assignment_id, stream_id).results)


class StreamingMediaTenantEngine(MicroserviceTenantEngine):
    def tenant_initialize(self, monitor):
        ds = self.config.get("datastore", {"type": "memory"})
        store = create_store(ds.get("type", "memory"), **{k: v for k, v in ds.items() if k != "type"})
        self.api = {"StreamingMedia": DeviceStreamManager(self, store)}


class StreamingMediaMicroservice(MultitenantMicroservice):
    identifier = "streaming-media"
    name = "Streaming Media"

    def service_names(self):
        return ["StreamingMedia"]

    def create_tenant_engine(self, tenant):
        return StreamingMediaTenantEngine(self, tenant)


# ============================================================================ event search
class SolrSearchProvider:
    def __init__(self, pid: str, url: str, collection: str = "SiteWhere", get=None):
        self.pid, self.url, self.collection = pid, url.rstrip("/"), collection
        self._get = get

    def search(self, query: str, rows: int = 100) -> list[dict]:
        url = f"{self.url}/{self.collection}/select?{urllib.parse.urlencode({'q': query, 'rows': rows, 'wt': 'json'})}"
        body = self._get(url) if self._get else urllib.request.urlopen(url, timeout=10).read()
        return json.loads(body).get("response", {}).get("docs", [])


class EventStoreSearchProvider:
    """In-process provider: ``field:value`` terms (AND) over the tenant's event store."""

    def __init__(self, pid: str, engine):
        self.pid, self._e = pid, engine

    def search(self, query: str, rows: int = 100) -> list[dict]:
        terms = dict(t.split(":", 1) for t in query.split() if ":" in t)
        em = self._e.ms.api("DeviceEventManagement", self._e.tenant.token)
        from ..models.domain import DateRangeSearchCriteria, DeviceEventType
        et = DeviceEventType(terms.pop("eventType", "Measurement"))
        idx = "Assignment"
        ids = []
        for k in ("assignment", "customer", "area", "asset"):
            if k in terms:
                idx, ids = k.title(), [terms.pop(k)]
        fn = {DeviceEventType.Measurement: em.list_measurements_for_index, DeviceEventType.Location: em.list_locations_for_index,
              DeviceEventType.Alert: em.list_alerts_for_index}.get(et, em.list_measurements_for_index)
        res = fn(idx, ids, DateRangeSearchCriteria(page_size=rows))
        out = []
        for ev in res.results:
            d = ev.to_dict()
            if all(str(d.get(k)) == v for k, v in terms.items()):
                out.append(d)
        return out


class SearchProviderManager:
    def __init__(self, providers: dict):
        self._p = providers

    def list_search_providers(self) -> list[dict]:
        return [{"id": k, "type": type(v).__name__} for k, v in self._p.items()]

    def search(self, provider_id: str, query: str, rows: int = 100) -> list[dict]:
        p = self._p.get(provider_id)
        if p is None:
            raise NotFoundException(ErrorCode.Error, f"search provider {provider_id}")
        return p.search(query, rows)


class EventSearchTenantEngine(MicroserviceTenantEngine):
    def tenant_initialize(self, monitor):
        prov = {"events": EventStoreSearchProvider("events", self)}
        for pc in self.config.get("providers", []):
            if pc.get("type") == "solr":
                prov[pc["id"]] = SolrSearchProvider(pc["id"], pc["url"], pc.get("collection", "SiteWhere"))
        self.api = {"EventSearch": SearchProviderManager(prov)}


class EventSearchMicroservice(MultitenantMicroservice):
    identifier = "event-search"
    name = "Event Search"

    def service_names(self):
        return ["EventSearch"]

    def create_tenant_engine(self, tenant):
        return EventSearchTenantEngine(self, tenant)
