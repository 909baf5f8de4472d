"""Import the reference's Spring XML tenant configuration into this framework's JSON documents.

A SiteWhere 2.x tenant is configured by one Spring XML file per multitenant service
(``service-tenant-management/dockerimage/templates/<template>/<service>.xml``), parsed there by
``*Parser`` classes against the ``*.xsd`` schemas.  Here a tenant is configured by
one JSON document per service (``services/tenant_management.TENANT_TEMPLATES``).  This module
converts the former into the latter so a reference deployment's templates can be brought over:

    python -m sitewhere_amd.runtime.xml_import /path/to/templates/default      # prints the JSON template

Coverage: every element used by the reference's five tenant templates (default, mongodb,
influxdb, cassandra, stomp) plus the common event-source, decoder, deduplicator, connector,
router and datastore elements of the schemas.  Anything not understood is reported in
``warnings`` rather than silently dropped.  The reference's Spring placeholders carry over:
``${tenant.token}`` / ``${tenant.id}`` become ``[[tenant.token]]`` / ``[[tenant.id]]`` and
``${prop:default}`` stays as is (resolved from the instance properties / environment).
"""
from __future__ import annotations

import copy
import json
import os
import re
import sys
import xml.etree.ElementTree as ET

_MONGO = {"type": "mongodb", "uri": "${mongodb.uri:mongodb://localhost:27017}", "database": "tenant-[[tenant.token]]"}
_CASSANDRA = {"type": "cassandra", "address": "${cassandra.address:}", "keyspace": "tenant_[[tenant.token]]",
              "bucket_ms": 3600000}
_INFLUX = {"type": "influxdb", "url": "${influxdb.url:http://localhost:8086}", "database": "tenant-[[tenant.token]]"}


def _local(tag: str) -> str:
    return tag.rsplit("}", 1)[-1]


def _sub(v: str | None) -> str | None:
    """Reference placeholders -> ours (tenant properties use the [[...]] form here)."""
    if v is None:
        return None
    return re.sub(r"\$\{tenant\.(token|id)\}", r"[[tenant.\1]]", v)


def _num(v, default=None):
    if v is None:
        return default
    v = _sub(v)
    try:
        return int(v)
    except ValueError:
        return v                           # a placeholder: resolved at tenant start


def _bool(v, default=None):
    return default if v is None else str(v).strip().lower() in ("true", "1", "yes")


def _period(v: str | None) -> str | None:
    """Reference durations (``10m``, ``8h``, ``1d``, ``30s``) -> ISO-8601 (``PT10M``)."""
    if not v:
        return None
    m = re.fullmatch(r"\s*(\d+)\s*([smhd])\s*", v.lower())
    if not m:
        return v
    n, u = m.groups()
    return f"P{n}D" if u == "d" else f"PT{n}{u.upper()}"


class _Ctx:
    def __init__(self):
        self.warnings: list[str] = []

    def warn(self, service: str, el: ET.Element):
        self.warnings.append(f"{service}: <{_local(el.tag)}> not imported")


def _datastore(el: ET.Element, ctx: _Ctx, service: str) -> dict | None:
    for c in el.iter():
        n = _local(c.tag)
        if n == "mongodb-datastore-reference":
            return dict(_MONGO)
        if n == "mongodb-datastore":
            host, port = _sub(c.get("hostname", "localhost")), _sub(c.get("port", "27017"))
            return {"type": "mongodb", "uri": f"mongodb://{host}:{port}",
                    "database": _sub(c.get("databaseName")) or "tenant-[[tenant.token]]"}
        if n == "cassandra-datastore-reference":
            return dict(_CASSANDRA)
        if n == "cassandra-datastore":
            return {**_CASSANDRA, "address": f"{_sub(c.get('contactPoints', 'localhost'))}:9042",
                    "keyspace": _sub(c.get("keyspace")) or _CASSANDRA["keyspace"]}
        if n == "influxdb-datastore-reference":
            return dict(_INFLUX)
        if n == "influxdb-datastore":
            return {**_INFLUX, "url": f"http://{_sub(c.get('hostname', 'localhost'))}:{_sub(c.get('port', '8086'))}",
                    "database": _sub(c.get("databaseName")) or _INFLUX["database"]}
    return None


# ------------------------------------------------------------------------------ event sources
_DECODERS = {"protobuf-event-decoder": "protobuf", "json-device-request-decoder": "json",
             "json-event-decoder": "json", "json-batch-event-decoder": "json-batch",
             "groovy-event-decoder": "script", "groovy-string-event-decoder": "script",
             "scripted-event-decoder": "script", "echo-string-decoder": "echo", "payload-logger-decoder": "echo",
             "coap-json-decoder": "coap-json", "composite-decoder": "composite", "composite-event-decoder": "composite"}


def _decoder(c: ET.Element):
    """A decoder element -> decoder spec: a name, or a dict for scripted / composite decoders
    (``composite-decoder``: ``groovy-device-metadata-extractor`` + ``choices`` of
    ``device-specification-decoder-choice token=...`` each wrapping a decoder)."""
    kind = _DECODERS[_local(c.tag)]
    if kind == "script":
        return {"type": "script", "script": _sub(c.get("scriptId") or c.get("scriptPath"))}
    if kind == "composite":
        spec: dict = {"type": "composite", "choices": {}}
        for x in c.iter():
            xn = _local(x.tag)
            if xn in ("groovy-device-metadata-extractor", "scripted-device-metadata-extractor"):
                spec["extractorScript"] = _sub(x.get("scriptId") or x.get("scriptPath"))
            elif xn == "device-specification-decoder-choice":
                inner = [d for d in x if _local(d.tag) in _DECODERS]
                if inner:
                    spec["choices"][_sub(x.get("token"))] = _decoder(inner[0])
        return spec
    return kind


def _mqtt_attrs(el: ET.Element) -> dict:
    """``cn:mqtt-broker-attributes`` (``connector-common.xsd``) of an MQTT receiver, connector or
    command destination: connection, credentials, trust / key stores, client id, session, QoS."""
    out = {"host": _sub(el.get("hostname", "localhost")), "port": _num(el.get("port"), 1883)}
    for k in ("protocol", "username", "password", "trustStorePath", "keyStorePath", "clientId", "cleanSession",
              "qos"):
        if el.get(k) is not None:
            out[k] = _sub(el.get(k))
    return out


def _receiver(n: str, el: ET.Element) -> dict | None:
    g = lambda k, d=None: _sub(el.get(k, d))   # noqa: E731
    if n == "mqtt-event-source":
        return dict(_mqtt_attrs(el), type="mqtt", topic=g("topic", "SiteWhere/input"),
                    numThreads=_num(el.get("numThreads"), 4))
    if n in ("activemq-event-source", "activemq-client-event-source"):
        if el.get("transportUri"):
            return {"type": "activemq-broker", "transportUri": g("transportUri"),
                    "queueName": g("queueName", "SITEWHERE.IN"), "numConsumers": _num(el.get("numConsumers"), 3),
                    "brokerName": g("brokerName")}
        host, port = "127.0.0.1", 61613
        m = re.match(r"^\w+://([^:/?]+)(?::(\d+))?", el.get("remoteUri") or "")
        if m:
            host, port = m.group(1), int(m.group(2) or 61613)
        return {"type": "activemq", "host": host, "port": port,
                "destination": "/queue/" + (g("queueName") or "SITEWHERE.IN"),
                "numThreads": _num(el.get("numConsumers"), 2)}
    if n == "rabbit-mq-event-source" or n == "rabbitmq-event-source":
        m = re.match(r"^amqps?://(?:[^@]*@)?([^:/]+)(?::(\d+))?", el.get("connectionUri") or "")
        return {"type": "rabbitmq", "host": m.group(1) if m else "127.0.0.1",
                "port": int(m.group(2) or 5672) if m else 5672, "queue": g("queueName", "sitewhere.input"),
                "durable": _bool(el.get("durable"), False)}
    if n == "socket-event-source":
        rc = {"type": "socket", "host": "0.0.0.0", "port": _num(el.get("port"), 8484),
              "numThreads": _num(el.get("numThreads"), 4), "handler": "read-all"}
        for c in el.iter():             # interaction handler factory (read-all / http / groovy)
            cn = _local(c.tag)
            if cn == "http-interaction-handler-factory":
                rc["handler"] = "http"
            elif cn in ("groovy-interaction-handler-factory", "groovy-socket-interaction-handler-factory"):
                rc.update(handler="script", script=_sub(c.get("scriptId") or c.get("scriptPath")))
        return rc
    if n in ("web-socket-event-source", "websocket-event-source"):
        rc = {"type": "websocket", "host": "0.0.0.0", "port": _num(el.get("port"), 8585),
              "payloadType": (g("payloadType") or "binary").lower()}
        if el.get("webSocketUrl"):
            rc["webSocketUrl"] = g("webSocketUrl")
        headers = {_sub(h.get("name")): _sub(h.get("value")) for h in el.iter() if _local(h.tag) == "header"}
        if headers:
            rc["headers"] = headers
        return rc
    if n == "coap-event-source" or n == "coap-server-event-source":
        return {"type": "coap", "host": g("hostname", "0.0.0.0"), "port": _num(el.get("port"), 5683)}
    if n in ("polling-rest-event-source", "rest-event-source"):
        ms = _num(el.get("pollIntervalMs"), 10000)
        rc = {"type": "rest-poll", "baseUrl": g("baseUrl") or g("url"),
              "interval": ms / 1000.0 if isinstance(ms, int) else 10.0}
        for k in ("username", "password"):
            if el.get(k):
                rc[k] = g(k)
        if el.get("scriptId"):
            rc["scriptId"] = g("scriptId")
        return rc
    if n in ("azure-eventhub-event-source", "eventhub-event-source"):
        ns, hub = g("namespace"), g("eventHubName") or g("targetFqn")
        return {"type": "eventhub", "namespace": ns, "eventHub": hub, "consumerGroup": g("consumerGroupName", "$Default"),
                "connectionString": f"Endpoint=sb://{ns}.servicebus.windows.net/;SharedAccessKeyName={g('sasKeyName')};"
                                    f"SharedAccessKey={g('sasKey')};EntityPath={hub}"}
    return None


def _event_sources(root: ET.Element, ctx: _Ctx) -> dict:
    sources, doc = [], {}
    for el in root.iter():
        n = _local(el.tag)
        if not n.endswith("-event-source"):
            if n in ("alternate-id-deduplicator",):
                doc["deduplicator"] = {"type": "alternate-id"}
            elif n in ("groovy-event-deduplicator", "scripted-event-deduplicator"):
                doc["deduplicator"] = {"type": "script", "script": _sub(el.get("scriptId") or el.get("scriptPath"))}
            continue
        rc = _receiver(n, el)
        if rc is None:
            ctx.warn("event-sources", el)
            continue
        src = {"id": _sub(el.get("sourceId")) or f"source-{len(sources) + 1}", "decoder": "json", "receivers": [rc]}
        for c in el:
            cn = _local(c.tag)
            if cn in _DECODERS:
                d = _decoder(c)
                if isinstance(d, dict) and d["type"] == "script":
                    src["decoder"], src["script"] = "script", d["script"]
                else:
                    src["decoder"] = d
            elif cn.endswith("-decoder") or cn.endswith("-event-decoder"):
                ctx.warn("event-sources", c)
        sources.append(src)
    doc["sources"] = sources
    return doc


# ------------------------------------------------------------------------------ other services
def _outbound(root: ET.Element, ctx: _Ctx) -> dict:
    out = []
    for el in root.iter():
        n = _local(el.tag)
        if not n.endswith("-connector"):
            continue
        g = lambda k, d=None: _sub(el.get(k, d))   # noqa: E731
        cid = g("connectorId") or f"connector-{len(out) + 1}"
        if n == "mqtt-connector":
            out.append(dict(_mqtt_attrs(el), id=cid, type="mqtt",
                            topic=g("outboundTopic") or g("topic", "SiteWhere/output")))
        elif n == "solr-connector":
            out.append({"id": cid, "type": "solr", "url": g("solrServerUrl") or g("url")})
        elif n in ("rabbit-mq-connector", "rabbitmq-connector"):
            m = re.match(r"^amqps?://(?:([^:@]*):?([^@]*)@)?([^:/]+)(?::(\d+))?", el.get("connectionUri") or "")
            rc = {"id": cid, "type": "rabbitmq", "exchange": g("exchange", ""),
                  "routingKey": g("topic") or "sitewhere.[[tenant.token]].events"}
            if m:
                rc.update(host=m.group(3), port=int(m.group(4) or 5672))
                if m.group(1):
                    rc.update(username=m.group(1), password=m.group(2))
            out.append(rc)
        elif n in ("aws-sqs-connector", "sqs-connector"):
            out.append({"id": cid, "type": "sqs", "queueUrl": g("queueUrl"), "accessKey": g("accessKey"),
                        "secretKey": g("secretKey"), "region": g("region")})
        elif n in ("azure-eventhub-connector", "eventhub-connector"):
            out.append({"id": cid, "type": "eventhub", "namespace": g("serviceBusNamespace") or g("namespace"),
                        "hub": g("eventHubName"), "sasKeyName": g("sasName"), "sasKey": g("sasKey")})
        elif n == "dweet-io-connector":
            out.append({"id": cid, "type": "dweet"})
        elif n == "initial-state-connector":
            out.append({"id": cid, "type": "initialstate", "accessKey": g("streamingAccessKey")})
        elif n in ("groovy-connector", "scripted-connector"):
            out.append({"id": cid, "type": "script", "script": g("scriptId") or g("scriptPath")})
        elif n == "http-connector":
            out.append({"id": cid, "type": "http", "url": g("url")})
        else:
            ctx.warn("outbound-connectors", el)
    return {"connectors": out}


def _rules(root: ET.Element, ctx: _Ctx) -> dict:
    procs = []
    for el in root.iter():
        n = _local(el.tag)
        if n == "zone-test-rule-processor" or n == "zone-test-processor":
            tests = [{"zoneToken": _sub(t.get("zoneToken")), "condition": t.get("condition", "inside"),
                      "alertType": _sub(t.get("alertType")), "alertLevel": t.get("alertLevel", "Warning"),
                      "alertMessage": _sub(t.get("alertMessage"))} for t in el if _local(t.tag) == "zone-test"]
            procs.append({"id": _sub(el.get("processorId")) or f"zones-{len(procs) + 1}", "type": "zone-test",
                          "zoneTests": tests})
        elif n in ("groovy-rule-processor", "scripted-rule-processor"):
            procs.append({"id": _sub(el.get("processorId")) or f"script-{len(procs) + 1}", "type": "script",
                          "script": _sub(el.get("scriptId") or el.get("scriptPath"))})
        elif n.endswith("-rule-processor") or n.endswith("-processor"):
            ctx.warn("rule-processing", el)
    return {"processors": procs}


def _command_delivery(root: ET.Element, ctx: _Ctx) -> dict:
    doc: dict = {"destinations": []}
    for el in root.iter():
        n = _local(el.tag)
        g = lambda k, d=None: _sub(el.get(k, d))   # noqa: E731
        if n.endswith("-command-destination"):
            enc = "json"
            for c in el:
                cn = _local(c.tag)
                if "protobuf" in cn:
                    enc = "protobuf"
                elif "json" in cn:
                    enc = "json"
            d = {"id": g("destinationId") or "default", "encoder": enc}
            if n == "mqtt-command-destination":
                d.update(_mqtt_attrs(el), provider="mqtt")
            elif n == "coap-command-destination":
                d.update(provider="coap")
            elif n in ("twilio-command-destination", "sms-command-destination"):
                d.update(provider="sms", accountSid=g("accountSid"), authToken=g("authToken"), fromPhone=g("fromPhoneNumber"))
            else:
                ctx.warn("command-delivery", el)
                continue
            doc["destinations"].append(d)
        elif n == "device-type-mapping-router":
            doc["router"] = {"type": "device-type-mapping", "default": g("defaultDestination"),
                             "mappings": {_sub(m.get("deviceTypeToken") or m.get("specification")): _sub(m.get("destination"))
                                          for m in el if _local(m.tag) == "mapping"}}
        elif n == "single-choice-command-router" or n == "single-choice-router":
            doc["router"] = {"type": "single-choice", "destination": g("destination")}
        elif n in ("groovy-command-router", "scripted-command-router"):
            doc["router"] = {"type": "script", "script": g("scriptId") or g("scriptPath")}
        elif n == "no-op-command-router":
            doc["router"] = {"type": "no-op"}
    if "router" in doc and doc["router"].get("type") == "device-type-mapping" and not doc["router"]["mappings"]:
        # a mapping router with no mappings routes everything to its default destination
        doc["router"] = {"type": "single-choice", "destination": doc["router"]["default"]}
    return doc


def _simple(service: str):
    def conv(root: ET.Element, ctx: _Ctx) -> dict:
        doc: dict = {}
        ds = _datastore(root, ctx, service)
        if ds is not None:
            doc["datastore"] = ds
            if service == "event-management" and ds["type"] in ("mongodb", "influxdb"):
                doc["buffered"] = True          # the reference's bulk buffer in front of Mongo / Influx
        for el in root.iter():
            n = _local(el.tag)
            if n == "inbound-processing":
                if el.get("processingThreadCount"):
                    doc["processingThreadCount"] = _num(el.get("processingThreadCount"))
            elif n == "presence-manager":
                doc["presence"] = {"checkInterval": _period(el.get("checkInterval")) or "PT10M",
                                   "missingInterval": _period(el.get("presenceMissingInterval")) or "PT8H"}
            elif n == "default-registration-manager":
                for k, ours in (("allowNewDevices", "allowNewDevices"), ("autoAssignSite", "autoAssign"),
                                ("autoAssign", "autoAssign")):
                    if el.get(k) is not None:
                        doc[ours] = _bool(el.get(k))
                for k in ("defaultDeviceTypeToken", "defaultCustomerToken", "defaultAreaToken"):
                    if el.get(k) is not None:
                        doc[k] = _sub(el.get(k))
            elif n == "qr-code-label-generator":
                doc.setdefault("generators", []).append({"id": _sub(el.get("id")) or "qrcode", "type": "qrcode"})
            elif n == "solr-search-provider":
                doc.setdefault("providers", []).append({"id": _sub(el.get("id")) or "solr", "type": "solr",
                                                        "url": _sub(el.get("solrServerUrl"))})
            elif n == "batch-operation-manager" and el.get("throttleDelayMs"):
                doc["throttleDelayMs"] = _num(el.get("throttleDelayMs"))
        return doc
    return conv


CONVERTERS = {"event-sources": _event_sources, "outbound-connectors": _outbound, "rule-processing": _rules,
              "command-delivery": _command_delivery}
SERVICES = ("asset-management", "batch-operations", "command-delivery", "device-management", "device-registration",
            "device-state", "event-management", "event-search", "event-sources", "inbound-processing",
            "label-generation", "outbound-connectors", "rule-processing", "schedule-management", "streaming-media")


def convert_service(service: str, xml: bytes | str, ctx: _Ctx | None = None) -> dict:
    """One reference ``<service>.xml`` -> this framework's configuration document."""
    ctx = ctx or _Ctx()
    root = ET.fromstring(xml)
    return CONVERTERS.get(service, _simple(service))(root, ctx)


def import_tenant_template(directory: str, base: dict | None = None) -> dict:
    """A reference template directory -> ``{"name", "services": {...}, "warnings": [...]}``.

    Services the directory does not configure keep ``base``; configured ones are deep-merged over
    it.  The reference's non-default templates (mongodb, influxdb, cassandra, stomp) are overlays
    of its ``default`` template, so by default a sibling ``default`` directory is imported first
    and used as the base; without one, this framework's ``default`` template is."""
    from ..services.tenant_management import TENANT_TEMPLATES
    from .config import deep_merge
    ctx = _Ctx()
    if base is None:
        sibling = os.path.join(os.path.dirname(os.path.normpath(directory)), "default")
        if os.path.basename(os.path.normpath(directory)) != "default" and os.path.isdir(sibling):
            ref_default = import_tenant_template(sibling)
            ctx.warnings += ref_default["warnings"]
            base = ref_default
        else:
            base = TENANT_TEMPLATES["default"]
    base = copy.deepcopy(base)
    name = os.path.basename(os.path.normpath(directory))
    meta = os.path.join(directory, "tenant-template.json")
    if os.path.exists(meta):
        with open(meta) as f:
            name = json.load(f).get("name", name).strip() or name
    services = base.get("services", {})
    for svc in SERVICES:
        p = os.path.join(directory, f"{svc}.xml")
        if not os.path.exists(p):
            continue
        with open(p, "rb") as f:
            doc = convert_service(svc, f.read(), ctx)
        if svc in ("event-sources", "outbound-connectors", "rule-processing"):
            merged = dict(services.get(svc, {}))
            merged.update(doc)                 # list-valued sections replace, not merge
            services[svc] = merged
        else:
            merged = deep_merge(services.get(svc, {}), doc)
            if "datastore" in doc:             # a different store type: none of the base store's keys apply
                merged["datastore"] = doc["datastore"]
            services[svc] = merged
    return {"name": f"{name} (imported)", "services": services, "warnings": ctx.warnings}


def register_reference_templates(root: str, prefix: str = "ref-") -> list[str]:
    """Import every template directory under ``root`` (the reference's
    ``service-tenant-management/dockerimage/templates``) as tenant template ``<prefix><dir>``."""
    from ..services.tenant_management import TENANT_TEMPLATES
    ids = []
    for d in sorted(os.listdir(root)):
        p = os.path.join(root, d)
        if os.path.isdir(p) and any(f.endswith(".xml") or f == "tenant-template.json" for f in os.listdir(p)):
            t = import_tenant_template(p)
            TENANT_TEMPLATES[prefix + d] = {"name": t["name"], "services": t["services"]}
            ids.append(prefix + d)
    return ids


def main(argv=None):
    argv = argv if argv is not None else sys.argv[1:]
    if not argv:
        print("usage: python -m sitewhere_amd.runtime.xml_import <reference template directory>", file=sys.stderr)
        return 2
    print(json.dumps(import_tenant_template(argv[0]), indent=2, sort_keys=True))
    return 0


if __name__ == "__main__":
    sys.exit(main())

