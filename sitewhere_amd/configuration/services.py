"""Models of the management, processing, delivery and platform services.

Reference: the ``*ModelProvider`` / ``*Roles`` pairs of service-event-management,
service-device-management, service-asset-management, service-batch-operations,
service-schedule-management, service-device-state, service-rule-processing,
service-outbound-connectors (``OutboundConnectorsModelProvider.java``: one element per connector,
filters and multicasters as child roles), service-command-delivery (``CommandDeliveryModelProvider``:
router, destinations with encoder / parameter extractor / delivery provider), service-label-generation,
service-streaming-media, service-event-search, service-instance-management,
service-tenant-management, service-user-management and service-web-rest.  Documents are the ones
the matching ``services/*.py`` modules read.
"""
from __future__ import annotations

from .common import DatastoreProvider, EventDatastoreProvider, FilterProvider, mqtt_attrs, script_attr
from .model import Attr, Element, ModelProvider, Role


class _DatastoreService(ModelProvider):
    """A multitenant service whose configuration is a datastore plus a few attributes."""

    attrs: tuple = ()
    children: tuple = ()

    def initialize_dependencies(self):
        self.dependencies = [DatastoreProvider()]

    def initialize_roles(self):
        self.role(Role(self.root_role, self.title, permanent=True, children=("datastore",) + tuple(self.children)))

    def initialize_elements(self):
        self.element(Element(self.title, self.root_role, (), self.description, list(self.attrs), icon="database"))


class DeviceManagementProvider(_DatastoreService):
    identifier = root_role = "device-management"
    title = "Device Management"
    description = "Device types, commands, statuses, devices, assignments, groups, customers, areas and zones."


class AssetManagementProvider(_DatastoreService):
    identifier = root_role = "asset-management"
    title = "Asset Management"
    description = "Asset types and assets."


class StreamingMediaProvider(_DatastoreService):
    identifier = root_role = "streaming-media"
    title = "Streaming Media"
    description = "Device streams and their chunks."


class UserManagementProvider(_DatastoreService):
    identifier = root_role = "user-management"
    title = "User Management"
    description = "Users, roles and granted authorities."


class TenantManagementProvider(_DatastoreService):
    identifier = root_role = "tenant-management"
    title = "Tenant Management"
    description = "Tenants and their configuration / dataset templates."


class BatchOperationsProvider(_DatastoreService):
    identifier = root_role = "batch-operations"
    title = "Batch Operations"
    description = "Batch command invocations and other operations over many devices."
    attrs = (Attr("threads", "Integer", "operation threads", default=10, group="perf"),
             Attr("throttleDelayMs", "Integer", "delay between elements", default=0, group="btch"))


class ScheduleManagementProvider(_DatastoreService):
    identifier = root_role = "schedule-management"
    title = "Schedule Management"
    description = "Cron / simple schedules and the jobs they trigger."
    attrs = (Attr("tickSeconds", "Decimal", "scheduler tick", default=1.0, group="perf"),)


class DeviceStateProvider(_DatastoreService):
    identifier = root_role = "device-state"
    title = "Device State"
    description = "Last-known state per assignment and presence detection."
    children = ("presence-manager",)

    def initialize_roles(self):
        super().initialize_roles()
        self.role(Role("presence-manager", "Presence Manager", key="presence"))

    def initialize_elements(self):
        super().initialize_elements()
        self.element(Element("Presence Manager", "presence-manager", (),
                             "Marks assignments missing after missingInterval (reference DevicePresenceManager).", [
                                 Attr("checkInterval", "String", "ISO-8601 period between checks", default="PT10M"),
                                 Attr("missingInterval", "String", "ISO-8601 period without events",
                                      default="PT8H")], icon="heartbeat"))


class EventManagementProvider(ModelProvider):
    identifier = root_role = "event-management"
    title = "Event Management"
    description = "Persist device events and publish persisted events."

    def initialize_dependencies(self):
        self.dependencies = [EventDatastoreProvider()]

    def initialize_roles(self):
        self.role(Role(self.root_role, self.title, permanent=True, children=("event-datastore",)))

    def initialize_elements(self):
        self.element(Element(self.title, self.root_role, (), self.description, [
            Attr("buffered", "Boolean", "bulk write buffer (reference DeviceEventBuffer)", default=False,
                 group="perf")], icon="database"))


class RuleProcessingProvider(ModelProvider):
    identifier = root_role = "rule-processing"
    title = "Rule Processing"
    description = "Rule processors run over enriched events."

    def initialize_roles(self):
        r = self.role
        r(Role(self.root_role, self.title, permanent=True, children=("rule-processor",)))
        r(Role("rule-processor", "Rule Processor", key="processors", multiple=True, reorderable=True))
        r(Role("zone-test", "Zone Test", key="zoneTests", multiple=True))
        r(Role("threshold-rule", "Threshold Rule", key="rules", multiple=True))

    def initialize_elements(self):
        e = self.element
        base = [Attr("id", "String", "processor id", required=True, index=True),
                Attr("numThreads", "Integer", "processing threads", default=0, group="perf")]
        e(Element(self.title, self.root_role, (), self.description, icon="cogs"))
        e(Element("Zone Test Processor", "rule-processor", ("zone-test",),
                  "Raise alerts when locations are inside / outside zones.", list(base), children=("zone-test",),
                  icon="map"))
        e(Element("Threshold Processor", "rule-processor", ("threshold",),
                  "Raise alerts when a measurement leaves [min, max].", list(base), children=("threshold-rule",),
                  icon="chart-line"))
        e(Element("Scripted Rule Processor", "rule-processor", ("script",),
                  "process(context, event, events_api, logger).", base + [script_attr()], icon="code"))
        level = Attr("alertLevel", "String", "alert level", default="Warning",
                     choices=("Info", "Warning", "Error", "Critical"))
        e(Element("Zone Test", "zone-test", (), "One geofence condition.", [
            Attr("zoneToken", "String", "zone", required=True),
            Attr("condition", "String", "inside | outside", default="inside", choices=("inside", "outside")),
            Attr("alertType", "String", "alert type", default="zone.alert"), level,
            Attr("alertMessage", "String", "alert message")], icon="map"))
        e(Element("Threshold Rule", "threshold-rule", (), "Bounds of one measurement.", [
            Attr("measurement", "String", "measurement name", required=True),
            Attr("min", "Decimal", "lower bound"), Attr("max", "Decimal", "upper bound"),
            Attr("alertType", "String", "alert type (default <name>.threshold)"), level,
            Attr("alertMessage", "String", "alert message")], icon="chart-line"))


class OutboundConnectorsProvider(ModelProvider):
    identifier = root_role = "outbound-connectors"
    title = "Outbound Connectors"
    description = "Forward enriched events to external systems."

    def initialize_dependencies(self):
        self.dependencies = [FilterProvider()]

    def initialize_roles(self):
        self.role(Role(self.root_role, self.title, permanent=True, children=("outbound-connector",)))
        self.role(Role("outbound-connector", "Outbound Connector", key="connectors", multiple=True,
                       children=("connector-filters",)))

    def initialize_elements(self):
        e = self.element
        base = [Attr("id", "String", "connector id", required=True, index=True),
                Attr("numProcessingThreads", "Integer", "processing threads", default=0, group="perf")]
        e(Element(self.title, self.root_role, (), self.description, icon="sign-out-alt"))

        def c(name, types, desc, attrs, icon="sign-out-alt"):
            e(Element(name, "outbound-connector", types, desc, base + attrs, icon=icon))
        c("Log Connector", ("log",), "Log every event.", [])
        c("MQTT Connector", ("mqtt",), "Publish each event to an MQTT topic.", [
            Attr("topic", "String", "topic template ({tenant}, {deviceToken})",
                 default="SiteWhere/{tenant}/outbound/{deviceToken}", group="conn"), *mqtt_attrs()])
        c("HTTP Connector", ("http",), "POST events as JSON.", [
            Attr("url", "String", "endpoint", required=True, group="conn"),
            Attr("headers", "Map", "request headers", group="conn"),
            Attr("batch", "Boolean", "one request per delivery batch", default=True, group="btch")])
        c("Solr Connector", ("solr",), "Index events in Apache Solr.", [
            Attr("url", "String", "Solr base URL", required=True, group="conn"),
            Attr("collection", "String", "collection", default="SiteWhere", group="conn")])
        c("File Archive Connector", ("file",), "Append events to JSON-lines files.", [
            Attr("path", "String", "archive directory", required=True, group="stor")])
        c("Scripted Connector", ("script",), "process(event, context).", [script_attr()], icon="code")
        c("Kafka Connector", ("kafka",), "Produce events to a Kafka topic.", [
            Attr("bootstrap", "String", "bootstrap servers", default="127.0.0.1:9092", group="conn"),
            Attr("topic", "String", "topic template", default="sitewhere.{tenant}.enriched", group="conn"),
            Attr("tls", "Boolean", "TLS", default=False, group="auth"),
            Attr("username", "String", "SASL PLAIN user", group="auth"),
            Attr("password", "String", "SASL PLAIN password", group="auth")])
        c("Amazon SQS Connector", ("sqs",), "Send events to an SQS queue (SigV4).", [
            Attr("queueUrl", "String", "queue URL", required=True, group="conn"),
            Attr("region", "String", "AWS region", default="us-east-1", group="conn"),
            Attr("accessKey", "String", "access key", required=True, group="auth"),
            Attr("secretKey", "String", "secret key", required=True, group="auth"),
            Attr("endpoint", "String", "endpoint override", group="conn")], icon="cloud")
        c("Azure EventHub Connector", ("eventhub",), "Send events to an Event Hub (SAS token).", [
            Attr("namespace", "String", "namespace", required=True, group="conn"),
            Attr("hub", "String", "event hub", required=True, group="conn"),
            Attr("sasKeyName", "String", "SAS key name", required=True, group="auth"),
            Attr("sasKey", "String", "SAS key", required=True, group="auth"),
            Attr("endpoint", "String", "endpoint override", group="conn")], icon="cloud")
        c("dweet.io Connector", ("dweet",), "Post events to dweet.io things.", [
            Attr("thing", "String", "thing name template", default="{deviceToken}", group="conn"),
            Attr("url", "String", "service URL", default="https://dweet.io", group="conn")], icon="cloud")
        c("RabbitMQ Connector", ("rabbitmq",), "Publish events to an AMQP exchange.", [
            Attr("host", "String", "broker host", default="127.0.0.1", group="conn"),
            Attr("port", "Integer", "AMQP port", default=5672, group="conn"),
            Attr("exchange", "String", "exchange", default="", group="conn"),
            Attr("routingKey", "String", "routing key template", default="sitewhere.{tenant}.events", group="conn"),
            Attr("username", "String", "user", default="guest", group="auth"),
            Attr("password", "String", "password", default="guest", group="auth"),
            Attr("vhost", "String", "virtual host", default="/", group="conn")])
        c("InitialState Connector", ("initialstate",), "Stream events to InitialState buckets.", [
            Attr("accessKey", "String", "access key", required=True, group="auth"),
            Attr("bucketKey", "String", "bucket key template", default="{deviceToken}", group="conn"),
            Attr("url", "String", "service URL", default="https://groker.init.st", group="conn")], icon="cloud")


class CommandDeliveryProvider(ModelProvider):
    identifier = root_role = "command-delivery"
    title = "Command Delivery"
    description = "Route command invocations to destinations that encode and deliver them."

    def initialize_roles(self):
        self.role(Role(self.root_role, self.title, permanent=True, children=("command-router", "command-destination")))
        self.role(Role("command-router", "Command Router", key="router"))
        self.role(Role("command-destination", "Command Destination", key="destinations", multiple=True,
                       discriminator="provider"))

    def initialize_elements(self):
        e = self.element
        e(Element(self.title, self.root_role, (), self.description, [
            Attr("processingThreads", "Integer", "delivery threads", default=5, group="perf")], icon="bolt"))
        e(Element("Single Choice Router", "command-router", ("single-choice",), "Every command to one destination.", [
            Attr("destination", "String", "destination id (default: the first)")], icon="random"))
        e(Element("Device Type Mapping Router", "command-router", ("device-type-mapping",),
                  "Destination chosen by the target's device type.", [
                      Attr("mappings", "Map", "device type token -> destination id", required=True),
                      Attr("default", "String", "destination when no mapping matches")], icon="random"))
        e(Element("Scripted Router", "command-router", ("script",),
                  "route(execution, gateway_token, assignment) -> destination id.", [script_attr()], icon="code"))
        e(Element("No-Op Router", "command-router", ("no-op",), "Drop every command.", icon="ban"))
        base = [Attr("id", "String", "destination id", required=True, index=True),
                Attr("encoder", "String", "command encoder", default="json", choices=("json", "protobuf", "script")),
                script_attr("encoderScript", "encode(execution, nesting, assignment) for encoder=script",
                            required=False)]
        e(Element("MQTT Command Destination", "command-destination", ("mqtt",),
                  "Publish encoded commands to per-device MQTT topics.", base + [
                      Attr("hostname", "String", "broker host (reference attribute name)", group="conn"),
                      Attr("commandTopic", "String", "command topic template",
                           default="SiteWhere/{tenant}/command/{deviceToken}", group="conn"),
                      Attr("systemTopic", "String", "system topic template",
                           default="SiteWhere/{tenant}/system/{deviceToken}", group="conn"), *mqtt_attrs()],
                  icon="sign-out-alt"))
        e(Element("CoAP Command Destination", "command-destination", ("coap",),
                  "Send commands to the device's CoAP endpoint (address from device metadata).", base + [
                      Attr("hostnameMetadata", "String", "metadata field of the host", default="coap_hostname"),
                      Attr("portMetadata", "String", "metadata field of the port", default="coap_port"),
                      Attr("urlMetadata", "String", "metadata field of the path", default="coap_url"),
                      Attr("methodMetadata", "String", "metadata field of the method", default="coap_method")],
                  icon="sign-out-alt"))
        e(Element("Twilio SMS Command Destination", "command-destination", ("sms",),
                  "Send commands as SMS through Twilio.", base + [
                      Attr("accountSid", "String", "account SID", group="auth"),
                      Attr("authToken", "String", "auth token", group="auth"),
                      Attr("fromPhone", "String", "sending number", group="conn"),
                      Attr("apiBase", "String", "API base URL", default="https://api.twilio.com", group="conn"),
                      Attr("phoneMetadata", "String", "metadata field of the device number", default="sms_phone")],
                  icon="sms"))
        e(Element("Log Command Destination", "command-destination", ("log",), "Log encoded commands.", base,
                  icon="file-alt"))


class LabelGenerationProvider(ModelProvider):
    identifier = root_role = "label-generation"
    title = "Label Generation"
    description = "Generate QR code labels for entities."

    def initialize_roles(self):
        self.role(Role(self.root_role, self.title, permanent=True, children=("label-generator",)))
        self.role(Role("label-generator", "Label Generator", key="generators", multiple=True))

    def initialize_elements(self):
        self.element(Element(self.title, self.root_role, (), self.description, icon="qrcode"))
        self.element(Element("QR Code Label Generator", "label-generator", ("qrcode",),
                             "QR code PNGs (encoder written from ISO/IEC 18004).", [
                                 Attr("id", "String", "generator id", required=True, index=True),
                                 Attr("ecLevel", "String", "error correction", default="M", choices=("L", "M", "Q", "H")),
                                 Attr("scale", "Integer", "pixels per module", default=6),
                                 Attr("baseUrl", "String", "encoded URL template")], icon="qrcode"))


class EventSearchProvider(ModelProvider):
    identifier = root_role = "event-search"
    title = "Event Search"
    description = "External search providers over stored events."

    def initialize_roles(self):
        self.role(Role(self.root_role, self.title, permanent=True, children=("search-provider",)))
        self.role(Role("search-provider", "Search Provider", key="providers", multiple=True))

    def initialize_elements(self):
        self.element(Element(self.title, self.root_role, (), self.description, icon="search"))
        self.element(Element("Solr Search Provider", "search-provider", ("solr",), "Query an Apache Solr collection.", [
            Attr("id", "String", "provider id", required=True, index=True),
            Attr("url", "String", "Solr base URL", required=True, group="conn"),
            Attr("collection", "String", "collection", default="SiteWhere", group="conn")], icon="search"))


class InstanceManagementProvider(ModelProvider):
    identifier = root_role = "instance-management"
    title = "Instance Management"
    description = "Instance bootstrap: configuration template, initial users and tenants."

    def initialize_roles(self):
        self.role(Role(self.root_role, self.title, permanent=True))

    def initialize_elements(self):
        self.element(Element(self.title, self.root_role, (), self.description, [
            Attr("instanceTemplate", "String", "instance template", default="default"),
            Attr("users", "List", "users created on bootstrap"),
            Attr("tenants", "List", "tenants created on bootstrap")], icon="server"))


class WebRestProvider(ModelProvider):
    identifier = root_role = "web-rest"
    title = "Web/REST"
    description = "REST API, JWT authentication and the admin UI."

    def initialize_roles(self):
        self.role(Role(self.root_role, self.title, permanent=True))

    def initialize_elements(self):
        self.element(Element(self.title, self.root_role, (), self.description, [
            Attr("port", "Integer", "HTTP port", default=8080, group="conn"),
            Attr("cors", "Boolean", "CORS", default=True, group="conn"),
            Attr("adminUiDir", "String", "directory of a built admin UI to serve")], icon="globe"))
