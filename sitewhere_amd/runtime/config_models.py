"""Configuration models (role / element trees) for every microservice.

Reference: each service's ``*ModelProvider`` + ``*Roles`` + ``*RoleKeys`` under
``sitewhere-configuration/.../configuration/model`` (``ConfigurationModelProvider.java:37-280``),
returned by the management RPC ``GetConfigurationModel`` so an editor can render and validate the
service's configuration.  Here the trees describe the JSON documents the services actually read
(``services/*.py`` ``self.config.get(...)``) and ``ConfigurationModel.validate`` checks them.
"""
from __future__ import annotations

from .config import AttributeNode as A
from .config import ConfigurationModel, ElementNode as E

DATASTORE = E("Datastore", "datastore", "Entity / event persistence backend", [
    A("type", "String", "memory | sqlite | mongodb | bucketed | influx | columnar", True, "memory",
      ["memory", "sqlite", "mongodb", "bucketed", "influx", "columnar"]),
    A("path", "String", "SQLite file (supports [[tenant.token]])"),
    A("uri", "String", "MongoDB connection URI (${mongodb.uri:...})"),
    A("database", "String", "database name"),
    A("bucket_ms", "Integer", "time bucket for the Cassandra-layout event store", default=3600000)])

MQTT_ATTRS = [
    A("protocol", "String", "tcp | ssl | tls", default="tcp", choices=["tcp", "ssl", "tls"]),
    A("username", "String", "MQTT user name"), A("password", "String", "MQTT password"),
    A("trustStorePath", "String", "PEM CA file for TLS (the reference's trust store)"),
    A("keyStorePath", "String", "PEM client certificate for mutual TLS (the reference's key store)"),
    A("keyPath", "String", "PEM client key (defaults to keyStorePath)"),
    A("clientId", "String", "MQTT client id"), A("cleanSession", "Boolean", "MQTT clean session", default=True),
    A("qos", "String", "0 | 1 | 2 or AT_MOST_ONCE | AT_LEAST_ONCE | EXACTLY_ONCE", default="1")]
DECODER = E("Decoder", "event-source-decoder", "Payload decoder", [
    A("type", "String", "protobuf | json | json-string | json-batch | coap-json | script | echo | composite", True, "json",
      ["protobuf", "json", "json-string", "json-batch", "coap-json", "script", "echo", "composite"]),
    A("script", "Script", "decoder script id or source (type=script)"),
    A("extractorScript", "Script", "composite: extract(payload, metadata) -> (deviceToken, payload)"),
    A("tokenField", "String", "composite without a script: JSON field holding the device token",
      default="deviceToken"),
    A("payloadField", "String", "composite without a script: JSON field holding the inner payload", default="payload")])
RECEIVER = E("Receiver", "event-source-receiver", "Protocol receiver", [
    A("type", "String", "mqtt | socket | websocket | coap | rest-poll | activemq | activemq-broker | rabbitmq | kafka | "
      "eventhub", True, choices=["mqtt", "socket", "websocket", "coap", "rest-poll", "activemq", "activemq-broker",
                                  "rabbitmq", "kafka", "eventhub"]),
    A("host", "String", "broker / bind host", default="127.0.0.1"), A("port", "Integer", "port"),
    A("topic", "String", "MQTT topic"), A("queue", "String", "AMQP queue"), A("destination", "String", "STOMP destination"),
    A("transportUri", "String", "embedded broker transport (activemq-broker), e.g. stomp://0.0.0.0:2345"),
    A("queueName", "String", "embedded broker queue (activemq-broker)"),
    A("numConsumers", "Integer", "embedded broker queue consumers", default=3),
    A("numThreads", "Integer", "processing threads", default=4),
    A("handler", "String", "socket interaction handler: read-all | line | http | script", default="read-all",
      choices=["read-all", "line", "http", "script"]),
    A("script", "Script", "socket interaction script interact(socket, receiver) / REST polling script "
      "poll(rest, payloads, logger)"),
    A("webSocketUrl", "String", "websocket: connect to this ws:// URL (client receiver) instead of listening"),
    A("payloadType", "String", "websocket: binary | string", default="binary", choices=["binary", "string"]),
    A("paths", "String", "coap: reference (devices/{token}/...) | any", default="reference",
      choices=["reference", "any"]),
    A("baseUrl", "String", "rest-poll: API base URL"), A("interval", "Double", "rest-poll: seconds", default=10.0),
    *MQTT_ATTRS])
SOURCE = E("Event Source", "event-source", "Decoder + deduplicator + receivers", [
    A("id", "String", "source id", True), A("decoder", "String", "decoder type or element", True),
    A("forward", "String", "'raw' forwards undecoded payload batches to the MI355X inbound engine"),
    A("logPayloads", "Boolean", "log every payload", default=False)], [DECODER, RECEIVER])

FILTER = E("Filter", "outbound-filter", "Event filter", [
    A("type", "String", "area | device-type | event-type | script", True),
    A("operation", "String", "include | exclude", default="include", choices=["include", "exclude"])])
CONNECTOR = E("Connector", "outbound-connector", "Outbound connector", [
    A("id", "String", "connector id", True),
    A("type", "String", "log | mqtt | http | solr | file | script | sqs | eventhub | dweet | initialstate | rabbitmq | kafka",
      True), A("numProcessingThreads", "Integer", "processing threads", default=0)], [FILTER])
PROCESSOR = E("Rule Processor", "rule-processor", "Rule processor", [
    A("id", "String", "processor id", True), A("type", "String", "zone-test | threshold | script", True),
    A("numThreads", "Integer", "processing threads", default=0)], [
    E("Zone Test", "zone-test", "Geofence test", [
        A("zoneToken", "String", "zone", True), A("condition", "String", "inside | outside", True, "inside"),
        A("alertType", "String", "alert type", True), A("alertLevel", "String", "Info | Warning | Error | Critical"),
        A("alertMessage", "String", "alert message")])])
DESTINATION = E("Command Destination", "command-destination", "Encoder + provider", [
    A("id", "String", "destination id", True), A("encoder", "String", "json | protobuf | script", True, "json"),
    A("provider", "String", "log | mqtt | coap | sms", True, "log"), A("host", "String", "MQTT host"),
    A("port", "Integer", "MQTT port"), A("commandTopic", "String", "MQTT command topic template"),
    A("accountSid", "String", "sms: Twilio account SID"), A("authToken", "String", "sms: Twilio auth token"),
    A("fromPhone", "String", "sms: sending number"), A("phoneMetadata", "String", "sms: device metadata field",
                                                          default="sms_phone"),
    A("hostnameMetadata", "String", "coap: device metadata field", default="coap_hostname"),
    A("portMetadata", "String", "coap: device metadata field", default="coap_port"),
    A("urlMetadata", "String", "coap: device metadata field", default="coap_url"),
    A("methodMetadata", "String", "coap: device metadata field", default="coap_method"),
    *MQTT_ATTRS])
ROUTER = E("Command Router", "command-router", "Destination choice", [
    A("type", "String", "single-choice | device-type-mapping | script | no-op", True, "single-choice"),
    A("destination", "String", "destination id (single-choice)")])

MODELS: dict[str, ConfigurationModel] = {}


def _m(identifier: str, title: str, attrs: list, children: list | None = None):
    MODELS[identifier] = ConfigurationModel(identifier, title, E(title, identifier, attributes=attrs,
                                                                 children=children or []))


_m("instance-management", "Instance Management", [A("instanceTemplate", "String", "instance template", True, "default")])
_m("user-management", "User Management", [], [DATASTORE])
_m("tenant-management", "Tenant Management", [], [DATASTORE])
_m("web-rest", "Web/REST", [A("port", "Integer", "HTTP port", default=8080), A("cors", "Boolean", "CORS", default=True)])
_m("event-sources", "Event Sources", [
    A("rawBatchSize", "Integer", "payloads per raw micro-batch (per partition) for the MI355X engine", default=4096),
    A("rawPartitioning", "Boolean", "split raw batches over the raw topic's partitions by device token "
      "(engine replicas own disjoint devices)", default=True),
    A("rawMaxDelayMs", "Integer", "latency bound of a raw micro-batch", default=5)], [SOURCE, E("Deduplicator", "deduplicator", "alternate-id | script", [
    A("type", "String", "alternate-id | script", True), A("script", "Script", "script id")])])
_m("inbound-processing", "Inbound Processing", [
    A("processingThreadCount", "Integer", "decoded-event processing threads", default=25),
    A("engine", "String", "cpu (per-event path) | gpu (fused MI355X micro-batch engine)", default="cpu",
      choices=["cpu", "gpu"]),
    A("device", "String", "gpu engine placement: auto | gpu | cpu", default="auto", choices=["auto", "gpu", "cpu"]),
    A("batchSize", "Integer", "micro-batch payloads (gpu engine)", default=65536),
    A("storage", "String", "objects | columnar (gpu engine)", default="objects", choices=["objects", "columnar"]),
    A("publishEnriched", "String", "events | batches | none (gpu engine)", default="events",
      choices=["events", "batches", "none"]),
    A("maxDelayMs", "Integer", "micro-batch latency bound (gpu engine)", default=5),
    A("gpuDevice", "Integer", "GPU of this replica (default SITEWHERE_GPU_DEVICE / LOCAL_RANK / 0)"),
    A("overlapSteps", "Boolean", "overlapped engine steps (default on for MI355X columnar tenants)"),
    A("asyncStore", "Boolean", "store rows on a store thread (default on for columnar storage)"),
    A("tuneGc", "Boolean", "freeze the start-up heap out of the cyclic GC", default=False),
    A("zeroCopyRows", "Boolean", "columnar payloads framed in place around the engine's pinned rows (pays with a bounded store window)", default=False)], [
    E("Zone Tests", "gpu-zone-tests", "zone tests evaluated inside the GPU engine", [
        A("zoneToken", "String", "zone", True), A("condition", "String", "inside | outside")]),
    E("Checkpoint", "checkpoint", "engine-shard snapshots; raw offsets commit only when covered", [
        A("path", "String", "safetensors file (supports [[tenant.token]])", True),
        A("everyBatches", "Integer", "raw batches between snapshots", default=64),
        A("includeStore", "Boolean", "also snapshot the HBM event ring", default=False)])])
_m("event-management", "Event Management", [A("buffered", "Boolean", "bulk buffer (DeviceEventBuffer)", default=False)],
   [DATASTORE])
_m("device-management", "Device Management", [], [DATASTORE])
_m("asset-management", "Asset Management", [], [DATASTORE])
_m("batch-operations", "Batch Operations", [A("threads", "Integer", "operation threads", default=10),
                                            A("throttleDelayMs", "Integer", "delay between elements", default=0)],
   [DATASTORE])
_m("schedule-management", "Schedule Management", [A("tickSeconds", "Decimal", "scheduler tick", default=1.0)], [DATASTORE])
_m("device-state", "Device State", [], [DATASTORE, E("Presence", "presence", "DevicePresenceManager", [
    A("checkInterval", "String", "ISO-8601 period", default="PT10M"),
    A("missingInterval", "String", "ISO-8601 period", default="PT8H")])])
_m("device-registration", "Device Registration", [
    A("allowNewDevices", "Boolean", "auto-register unknown devices", default=True),
    A("defaultDeviceTypeToken", "String", "device type for new devices"),
    A("defaultCustomerToken", "String", "customer for new assignments"),
    A("defaultAreaToken", "String", "area for new assignments"),
    A("autoAssign", "Boolean", "create an assignment on registration", default=True)])
_m("rule-processing", "Rule Processing", [], [PROCESSOR])
_m("outbound-connectors", "Outbound Connectors", [], [CONNECTOR])
_m("command-delivery", "Command Delivery", [A("processingThreads", "Integer", "delivery threads", default=5)],
   [ROUTER, DESTINATION])
_m("label-generation", "Label Generation", [], [E("Generator", "label-generator", "QR code generator", [
    A("id", "String", "generator id", True), A("type", "String", "qrcode", True, "qrcode"),
    A("ecLevel", "String", "L | M | Q | H", default="M"), A("scale", "Integer", "pixels per module", default=6),
    A("baseUrl", "String", "encoded URL template")])])
_m("streaming-media", "Streaming Media", [], [DATASTORE])
_m("event-search", "Event Search", [], [E("Search Provider", "search-provider", "external search provider", [
    A("id", "String", "provider id", True), A("type", "String", "solr", True), A("url", "String", "Solr base URL"),
    A("collection", "String", "collection", default="SiteWhere")])])


def model_for(identifier: str) -> ConfigurationModel | None:
    return MODELS.get(identifier)
