"""Models of the ingest services: event sources, inbound processing, device registration.

Reference: ``service-event-sources/.../configuration/EventSourcesModelProvider.java`` +
``EventSourcesRoles.java`` (event source -> decoder / deduplicator / receiver roles; one element per
receiver protocol and decoder; ``specializes`` restricting decoders per source kind),
``service-inbound-processing/.../InboundProcessingModelProvider.java`` and
``service-device-registration/.../DeviceRegistrationModelProvider.java``.  Documents are the ones
``services/event_sources.py``, ``edges/receivers.py:build_receiver``, ``services/gpu_inbound.py``
and ``services/device_registration.py`` read.
"""
from __future__ import annotations

from .common import mqtt_attrs, script_attr
from .model import Attr, Element, ModelProvider, Role

THREADS = Attr("numThreads", "Integer", "payload processing threads", default=4, group="perf")
HOST = Attr("host", "String", "bind / broker host", default="127.0.0.1", group="conn")


class EventSourcesProvider(ModelProvider):
    identifier, title, root_role = "event-sources", "Event Sources", "event-sources"
    description = "Receive payloads over device protocols, decode them and publish decoded / raw events."

    def initialize_roles(self):
        r = self.role
        r(Role("event-sources", "Event Sources", children=("event-source", "event-deduplicator"), permanent=True))
        r(Role("event-source", "Event Source", key="sources", multiple=True, reorderable=True,
               children=("event-decoder", "source-deduplicator", "event-receiver")))
        r(Role("event-decoder", "Event Decoder", key="decoder", optional=False, shorthand=True,
               subtypes=("binary-event-decoder", "string-event-decoder", "coap-event-decoder")))
        r(Role("binary-event-decoder", "Binary Event Decoder", key="decoder", shorthand=True,
               subtypes=("composite-event-decoder",)))
        r(Role("string-event-decoder", "String Event Decoder", key="decoder", shorthand=True))
        r(Role("coap-event-decoder", "CoAP Event Decoder", key="decoder", shorthand=True))
        r(Role("composite-event-decoder", "Composite Event Decoder", key="decoder",
               children=("composite-default-decoder",)))
        r(Role("composite-default-decoder", "Default Decoder", key="default", shorthand=True,
               subtypes=("binary-event-decoder",)))
        r(Role("event-deduplicator", "Event Deduplicator", key="deduplicator"))
        r(Role("source-deduplicator", "Source Deduplicator", key="deduplicator", subtypes=("event-deduplicator",)))
        r(Role("event-receiver", "Event Receiver", key="receivers", multiple=True,
               children=("websocket-headers",)))
        r(Role("websocket-headers", "WebSocket Headers", key="headers"))

    def initialize_elements(self):
        e = self.element
        e(Element("Event Sources", "event-sources", (), self.description, [
            Attr("rawBatchSize", "Integer", "payloads per raw micro-batch (per partition) for the MI355X engine",
                 default=4096, group="engn"),
            Attr("rawPartitioning", "Boolean", "split raw batches over the raw topic's partitions by device token "
                 "(engine replicas own disjoint devices)", default=True, group="engn"),
            Attr("rawMaxDelayMs", "Integer", "latency bound of a raw micro-batch", default=5, group="engn")],
            icon="sign-in-alt"))
        e(Element("Event Source", "event-source", (), "One decoder, an optional deduplicator and its receivers.", [
            Attr("id", "String", "unique source id", required=True, index=True),
            Attr("forward", "String", "'raw' forwards undecoded payload batches to the MI355X inbound engine "
                 "(JSON device requests are transcoded to protobuf natively; the rest keep the per-event path)",
                 choices=("raw",), group="engn"),
            Attr("logPayloads", "Boolean", "log every payload", default=False),
            Attr("script", "Script", "decoder script when decoder is 'script' (shorthand)", group="scrp")],
            icon="sign-in-alt"))
        # decoders
        e(Element("Protobuf Event Decoder", "binary-event-decoder", ("protobuf",),
                  "Reference sitewhere.proto device messages (GPU-decoded on raw-forwarding sources).",
                  icon="cogs"))
        e(Element("JSON Device Request Decoder", "binary-event-decoder", ("json",),
                  "One JSON device request per payload.", icon="cogs"))
        e(Element("JSON Batch Event Decoder", "binary-event-decoder", ("json-batch",),
                  "A JSON document carrying measurements / locations / alerts lists for one device.", icon="cogs"))
        e(Element("Scripted Event Decoder", "binary-event-decoder", ("script",),
                  "decode(payload, metadata) -> list of device requests.", [script_attr()], icon="code"))
        e(Element("Composite Event Decoder", "composite-event-decoder", ("composite",),
                  "Extract the device token, then decode with the decoder chosen for its device type.", [
                      script_attr("extractorScript", "extract(payload, metadata) -> (deviceToken, payload)",
                                  required=False),
                      Attr("tokenField", "String", "JSON field holding the device token (no script)",
                           default="deviceToken"),
                      Attr("payloadField", "String", "JSON field holding the inner payload (no script)",
                           default="payload"),
                      Attr("choices", "Map", "device type token -> decoder")], icon="sitemap"))
        e(Element("JSON String Event Decoder", "string-event-decoder", ("json-string",),
                  "JSON device request carried as text.", icon="cogs"))
        e(Element("Echo String Event Decoder", "string-event-decoder", ("echo",),
                  "Logs the payload (debugging).", icon="cogs"))
        e(Element("CoAP JSON Event Decoder", "coap-event-decoder", ("coap-json",),
                  "JSON bodies addressed by the CoAP resource path (devices/{token}/measurements ...).",
                  icon="cogs"))
        # deduplicators
        e(Element("Alternate Id Deduplicator", "event-deduplicator", ("alternate-id",),
                  "Drops a request whose alternate id event management already stored.", icon="copy"))
        e(Element("Scripted Deduplicator", "event-deduplicator", ("script",),
                  "is_duplicate(request) -> bool.", [script_attr()], icon="code"))
        # receivers
        e(Element("MQTT Event Source", "event-receiver", ("mqtt",), "Subscribe to an MQTT topic.", [
            Attr("hostname", "String", "broker host (reference attribute name)", group="conn"),
            Attr("topic", "String", "MQTT topic", default="SiteWhere/input", group="conn"),
            THREADS, *mqtt_attrs()], icon="sign-in-alt"))
        e(Element("Socket Event Source", "event-receiver", ("socket",), "Accept TCP connections.", [
            HOST, Attr("port", "Integer", "listen port", default=0, group="conn"), THREADS,
            Attr("handler", "String", "socket interaction handler", default="read-all",
                 choices=("read-all", "line", "http", "script")),
            script_attr(description="interact(socket, receiver) for handler=script", required=False)],
            icon="plug"))
        e(Element("WebSocket Event Source", "event-receiver", ("websocket",),
                  "Listen for WebSocket clients, or connect to webSocketUrl.", [
                      HOST, Attr("port", "Integer", "listen port", default=0, group="conn"),
                      Attr("webSocketUrl", "String", "connect to this ws:// URL instead of listening", group="conn"),
                      Attr("url", "String", "alias of webSocketUrl", group="conn"),
                      Attr("payloadType", "String", "binary | string", default="binary",
                           choices=("binary", "string"))], icon="plug"))
        e(Element("WebSocket Headers", "websocket-headers", (), "Headers sent on connect.", open=True))
        e(Element("CoAP Server Event Source", "event-receiver", ("coap",), "CoAP server (RFC 7252).", [
            HOST, Attr("port", "Integer", "UDP port", default=0, group="conn"),
            Attr("paths", "String", "reference resource tree or any path", default="reference",
                 choices=("reference", "any"))], icon="plug"))
        e(Element("Polling REST Event Source", "event-receiver", ("rest-poll",),
                  "Poll a REST API on an interval; a script turns responses into payloads.", [
                      Attr("baseUrl", "String", "API base URL", group="conn"),
                      Attr("url", "String", "alias of baseUrl", group="conn"),
                      Attr("interval", "Decimal", "seconds between polls", default=10.0, group="perf"),
                      Attr("headers", "Map", "request headers", group="conn"),
                      Attr("username", "String", "basic-auth user", group="auth"),
                      Attr("password", "String", "basic-auth password", group="auth"),
                      script_attr(description="poll(rest, payloads, logger)", required=False),
                      Attr("scriptId", "String", "script id of the polling script", group="scrp")],
                  icon="sync"))
        e(Element("ActiveMQ Broker Event Source", "event-receiver", ("activemq-broker",),
                  "Embedded STOMP broker with a consumer pool on one queue.", [
                      Attr("transportUri", "String", "stomp://host:port", default="stomp://127.0.0.1:61613",
                           group="conn"),
                      Attr("queueName", "String", "queue", default="SITEWHERE.IN", group="conn"),
                      Attr("numConsumers", "Integer", "queue consumers", default=3, group="perf"),
                      Attr("brokerName", "String", "broker name")], icon="sign-in-alt"))
        e(Element("ActiveMQ Client Event Source", "event-receiver", ("activemq", "stomp"),
                  "Consume a remote broker destination over STOMP.", [
                      HOST, Attr("port", "Integer", "STOMP port", default=61613, group="conn"),
                      Attr("destination", "String", "destination", default="/queue/SITEWHERE.IN", group="conn"),
                      Attr("transportUri", "String", "embedded broker transport instead of a client", group="conn"),
                      Attr("queueName", "String", "embedded broker queue", group="conn"),
                      Attr("numConsumers", "Integer", "embedded broker consumers", default=3, group="perf"),
                      Attr("login", "String", "STOMP login", group="auth"),
                      Attr("passcode", "String", "STOMP passcode", group="auth"),
                      Attr("numThreads", "Integer", "processing threads", default=2, group="perf")],
                  icon="sign-in-alt"))
        e(Element("RabbitMQ Event Source", "event-receiver", ("rabbitmq", "amqp"), "Consume an AMQP 0-9-1 queue.", [
            HOST, Attr("port", "Integer", "AMQP port", default=5672, group="conn"),
            Attr("queue", "String", "queue", default="sitewhere.input", group="conn"),
            Attr("username", "String", "user", default="guest", group="auth"),
            Attr("password", "String", "password", default="guest", group="auth"),
            Attr("vhost", "String", "virtual host", default="/", group="conn"),
            Attr("durable", "Boolean", "durable queue", default=False, group="conn")], icon="sign-in-alt"))
        e(Element("Kafka Event Source", "event-receiver", ("kafka",), "Consume a Kafka topic (wire protocol).", [
            Attr("bootstrap", "String", "bootstrap servers", default="127.0.0.1:9092", group="conn"),
            Attr("topic", "String", "topic", required=True, group="conn"),
            Attr("group", "String", "consumer group", default="sitewhere", group="conn"),
            Attr("tls", "Boolean", "TLS", default=False, group="auth"),
            Attr("username", "String", "SASL PLAIN user", group="auth"),
            Attr("password", "String", "SASL PLAIN password", group="auth")], icon="sign-in-alt"))
        e(Element("Azure EventHub Event Source", "event-receiver", ("eventhub", "azure-eventhub"),
                  "Consume every partition of an Event Hub over AMQP 1.0 (EventProcessorHost: partition leases "
                  "balanced over hosts, offsets checkpointed per consumer group), or over its Kafka endpoint.", [
                      Attr("protocol", "String", "amqp (SAS key) | kafka (connection string)", default="amqp",
                           choices=("amqp", "kafka"), group="conn"),
                      Attr("namespace", "String", "Event Hubs namespace", group="conn"),
                      Attr("host", "String", "endpoint host (default <namespace>.servicebus.windows.net)",
                           group="conn"),
                      Attr("port", "Integer", "AMQP port", default=5671, group="conn"),
                      Attr("bootstrap", "String", "kafka: host:port (default <namespace>.servicebus.windows.net:9093)",
                           group="conn"),
                      Attr("eventHub", "String", "event hub name", required=True, group="conn"),
                      Attr("consumerGroup", "String", "consumer group", default="$Default", group="conn"),
                      Attr("sasKeyName", "String", "amqp: shared access key name", group="auth"),
                      Attr("sasKey", "String", "amqp: shared access key", group="auth"),
                      Attr("connectionString", "String", "kafka: namespace connection string", group="auth"),
                      Attr("tls", "Boolean", "TLS", default=True, group="auth"),
                      Attr("hostNamePrefix", "String", "prefix of this host's lease owner name", default="sitewhere"),
                      Attr("partitionCount", "Integer", "partitions (default: asked from $management)"),
                      Attr("checkpointEvery", "Integer", "events between partition checkpoints", default=100,
                           group="perf")], icon="cloud"))


class InboundProcessingProvider(ModelProvider):
    identifier, title, root_role = "inbound-processing", "Inbound Processing", "inbound-processing"
    description = "Validate decoded events against the registry, persist them and publish enriched events."

    def initialize_roles(self):
        self.role(Role("inbound-processing", "Inbound Processing", permanent=True,
                       children=("engine-capacity", "gpu-zone-tests", "engine-checkpoint")))
        self.role(Role("engine-capacity", "Engine Capacity", key="capacity"))
        self.role(Role("gpu-zone-tests", "Zone Tests", key="zoneTests", multiple=True))
        self.role(Role("engine-checkpoint", "Checkpoint", key="checkpoint"))

    def initialize_elements(self):
        g = "engn"
        self.element(Element("Inbound Processing", "inbound-processing", (), self.description, [
            Attr("processingThreadCount", "Integer", "decoded-event processing threads", default=25, group="perf"),
            Attr("maxThreads", "Integer", "alias of processingThreadCount", group="perf"),
            Attr("engine", "String", "cpu (per-event path) | gpu (fused MI355X micro-batch engine)", default="cpu",
                 choices=("cpu", "gpu")),
            Attr("device", "String", "engine placement", default="auto", choices=("auto", "gpu", "cpu"), group=g),
            Attr("gpuDevice", "Integer", "GPU of this replica (default SITEWHERE_GPU_DEVICE / LOCAL_RANK / 0)",
                 group=g),
            Attr("cpuThreads", "Integer", "native CPU engine threads (device=cpu)", group=g),
            Attr("batchSize", "Integer", "micro-batch payloads", default=65536, group=g),
            Attr("maxDelayMs", "Integer", "micro-batch latency bound", default=5, group=g),
            Attr("sizing", "String", "small (capacity overrides EngineConfig.small) | full", default="small",
                 choices=("small", "full"), group=g),
            Attr("storage", "String", "where the engine's rows go", default="objects",
                 choices=("objects", "columnar", "durable"), group="stor"),
            Attr("publishEnriched", "String", "enriched output", default="events",
                 choices=("events", "batches", "none")),
            Attr("overlapSteps", "Boolean", "overlapped engine steps (default on for MI355X columnar tenants)",
                 group="perf"),
            Attr("asyncStore", "Boolean", "store rows on a store thread (default on for columnar storage)",
                 group="perf"),
            Attr("zeroCopyRows", "Boolean", "columnar payloads framed in place around the engine's pinned rows",
                 default=False, group="perf"),
            Attr("coalesceRaw", "Boolean", "step raw records already waiting in a partition together (up to "
                 "the engine's batch capacity; overlapped steps)", default=True, group="perf"),
            Attr("retainHostAllocations", "Boolean", "keep pinned host pools between steps", default=True,
                 group="perf"),
            Attr("tuneGc", "Boolean", "freeze the start-up heap out of the cyclic GC", default=False, group="perf"),
            Attr("rawBackpressure", "Boolean", "producers wait instead of retention dropping unread raw batches",
                 default=True, group="perf"),
            Attr("rawBackpressureWaitS", "Decimal", "longest producer wait before BackpressureTimeout",
                 default=60, group="perf"),
            Attr("presenceMissingMs", "Integer", "presence: missing after this long", group=g),
            Attr("presenceCheckMs", "Integer", "presence: check interval", group=g)], icon="cogs"))
        caps = [Attr(k, "Integer", d, group="engn") for k, d in (
            ("max_msgs", "payloads per micro-batch"), ("rec_cap", "decoded events per micro-batch"),
            ("gen_cap", "rule alerts + presence events per step"), ("max_devices", "registry capacity"),
            ("max_assignments", "assignment capacity"), ("store_cap", "HBM event ring (events)"),
            ("dedup_slots", "alternate-id window slots per generation"),
            ("dedup_filter_ids", "store-backed dedup filter: ids per generation (0 = off; ~8 B of HBM per id and generation)"),
            ("dedup_filter_gens", "store-backed dedup filter generations (2..8; the newest gens - 1 are always held)"),
            ("name_slots", "distinct names"),
            ("state_slots", "(assignment, name) state slots"), ("names_cap", "new-name reports per step"),
            ("shuffle_pad", "records added to every re-key slab"), ("carry_cap", "re-key carry records"),
            ("carry_high", "carry level that stalls new input"), ("presence_missing_ms", "presence missing"),
            ("presence_check_ms", "presence check"))]
        caps.append(Attr("shuffle_slack", "Decimal", "per-destination slab slack", group="engn"))
        self.element(Element("Engine Capacity", "engine-capacity", (),
                             "EngineConfig overrides sized for HBM (pipeline/config.py).", caps, icon="memory"))
        self.element(Element("Zone Test", "gpu-zone-tests", (), "Geofence evaluated inside the GPU engine.", [
            Attr("zoneToken", "String", "zone", required=True),
            Attr("condition", "String", "inside | outside", default="inside", choices=("inside", "outside")),
            Attr("alertType", "String", "alert type", default="zone.alert"),
            Attr("alertLevel", "Integer", "0 Info .. 3 Critical", default=1),
            Attr("alertMessage", "String", "alert message")], icon="map"))
        self.element(Element("Checkpoint", "engine-checkpoint", (),
                             "Engine-shard snapshots; raw offsets commit only when covered.", [
                                 Attr("path", "String", "safetensors file (supports [[tenant.token]])", required=True,
                                      group="stor"),
                                 Attr("everyBatches", "Integer", "raw batches between snapshots", default=64),
                                 Attr("includeStore", "Boolean", "also snapshot the HBM event ring", default=False)],
                             icon="save"))


class DeviceRegistrationProvider(ModelProvider):
    identifier, title, root_role = "device-registration", "Device Registration", "device-registration"
    description = "Register devices that send events before they exist (reference DefaultRegistrationManager)."

    def initialize_roles(self):
        self.role(Role("device-registration", "Device Registration", permanent=True))

    def initialize_elements(self):
        self.element(Element("Device Registration", "device-registration", (), self.description, [
            Attr("allowNewDevices", "Boolean", "auto-register unknown devices", default=True),
            Attr("defaultDeviceTypeToken", "String", "device type for new devices"),
            Attr("defaultCustomerToken", "String", "customer for new assignments"),
            Attr("defaultAreaToken", "String", "area for new assignments"),
            Attr("autoAssign", "Boolean", "create an assignment on registration", default=True)], icon="user-plus"))
