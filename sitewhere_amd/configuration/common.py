"""Shared roles and elements: datastores, MQTT connectivity, event filters, scripts.

Reference: ``sitewhere-configuration/.../model/CommonDatastoreRoles.java`` / ``CommonDatastoreProvider``
(MongoDB, InfluxDB, Cassandra datastore elements shared by every persistent service),
``CommonConnectorModel.addMqttCommonAttributes`` (protocol, host, port, TLS stores, credentials,
QoS) and ``CommonConnectorRoles`` (filters of outbound connectors).  The datastore elements here
are the stores ``persistence/store.py:create_store`` and ``persistence/events.py:create_event_store``
build; each microservice provider lists these providers as dependencies.
"""
from __future__ import annotations

from .model import Attr, Element, ModelProvider, Role


def mqtt_attrs(host_key: str = "host", port_default: int = 1883) -> list:
    """MQTT connectivity + authentication (reference CommonConnectorModel.addMqttCommonAttributes)."""
    return [
        Attr("protocol", "String", "tcp | ssl | tls", default="tcp", choices=("tcp", "ssl", "tls"), group="conn"),
        Attr(host_key, "String", "broker host", default="127.0.0.1", group="conn"),
        Attr("port", "Integer", "broker port", default=port_default, group="conn"),
        Attr("trustStorePath", "String", "PEM CA file for TLS (the reference's trust store)", group="auth"),
        Attr("trustStorePassword", "String", "unused with PEM trust stores", group="auth"),
        Attr("keyStorePath", "String", "PEM client certificate for mutual TLS (the reference's key store)",
             group="auth"),
        Attr("keyStorePassword", "String", "unused with PEM key stores", group="auth"),
        Attr("keyPath", "String", "PEM client key (defaults to keyStorePath)", group="auth"),
        Attr("username", "String", "MQTT user name", group="auth"),
        Attr("password", "String", "MQTT password", group="auth"),
        Attr("clientId", "String", "MQTT client id", group="conn"),
        Attr("cleanSession", "Boolean", "MQTT clean session", default=True, group="conn"),
        Attr("qos", "StringOrInteger", "0 | 1 | 2 or AT_MOST_ONCE | AT_LEAST_ONCE | EXACTLY_ONCE", default=1,
             group="conn")]


def script_attr(name: str = "script", description: str = "script id (script management) or inline source",
                required: bool = True) -> Attr:
    return Attr(name, "Script", description, required=required, group="scrp")


class DatastoreProvider(ModelProvider):
    """Entity datastores (device / asset / batch / schedule / state / media / user / tenant)."""

    def initialize_roles(self):
        self.role(Role("datastore", "Datastore", key="datastore", optional=True))

    def initialize_elements(self):
        self.element(Element("In-Memory Datastore", "datastore", ("memory",),
                             "Entities held in process memory (tests, single-node demos).", icon="memory"))
        self.element(Element("SQLite Datastore", "datastore", ("sqlite",),
                             "Entities in a SQLite file with indexed query columns.", [
                                 Attr("path", "String", "database file (supports [[tenant.token]]); ':memory:' "
                                      "keeps it in memory", default=":memory:", group="stor")], icon="database"))
        self.element(Element("MongoDB Datastore", "datastore", ("mongodb", "mongo"),
                             "Entities in MongoDB (reference MongoDB datastore), queries pushed down into find().", [
                                 Attr("uri", "String", "connection URI (${mongodb.uri:...})",
                                      default="mongodb://localhost:27017", group="conn"),
                                 Attr("database", "String", "database name", default="sitewhere", group="stor")],
                             icon="database"))


class EventDatastoreProvider(ModelProvider):
    """Event stores of event management (reference CommonDatastoreProvider + the MI355X stores)."""

    def initialize_roles(self):
        self.role(Role("event-datastore", "Event Datastore", key="datastore", optional=True))

    def initialize_elements(self):
        e = self.element
        e(Element("In-Memory Event Store", "event-datastore", ("memory",), "Events in process memory.", icon="memory"))
        e(Element("SQLite Event Store", "event-datastore", ("sqlite",), "Events in SQLite.", [
            Attr("path", "String", "database file (supports [[tenant.token]])", default=":memory:", group="stor")]))
        e(Element("MongoDB Event Store", "event-datastore", ("mongodb", "mongo"),
                  "Reference MongoDB layout: one events collection, compound indexes per index.", [
                      Attr("uri", "String", "connection URI", default="mongodb://localhost:27017", group="conn"),
                      Attr("database", "String", "database name", default="sitewhere", group="stor")]))
        e(Element("Apache Cassandra Event Store", "event-datastore", ("cassandra",),
                  "Reference Cassandra layout (events by id / assignment / customer / area / asset, time "
                  "buckets) over the CQL native protocol; no address: the in-process bucketed store.", [
                      Attr("address", "String", "contact point host[:port]", group="conn"),
                      Attr("keyspace", "String", "keyspace (supports [[tenant.token]])", default="sitewhere",
                           group="stor"),
                      Attr("bucket_ms", "Integer", "time bucket length", default=3600000, group="stor"),
                      Attr("username", "String", "CQL user", group="auth"),
                      Attr("password", "String", "CQL password", group="auth")]))
        e(Element("Bucketed Event Store", "event-datastore", ("bucketed",),
                  "In-process store with the Cassandra time-bucket layout.", [
                      Attr("bucket_ms", "Integer", "time bucket length", default=3600000, group="stor")]))
        e(Element("InfluxDB Event Store", "event-datastore", ("influxdb",),
                  "Events as InfluxDB points (line protocol writes, InfluxQL reads).", [
                      Attr("url", "String", "InfluxDB base URL", default="http://localhost:8086", group="conn"),
                      Attr("database", "String", "database", default="sitewhere", group="stor")]))
        e(Element("Columnar Event Store", "event-datastore", ("columnar",),
                  "MI355X engine rows held columnar in host memory (volatile; benchmarks of the pipeline).", [
                      Attr("retentionRows", "Integer", "rows kept before the oldest are evicted", group="stor")]))
        e(Element("Durable Segment Event Store", "event-datastore", ("segments", "durable"),
                  "MI355X engine rows as GPU-encoded column blocks in append-only segment files "
                  "(group-commit fdatasync, commit records for exactly-once ingest).", [
                      Attr("path", "String", "segment directory (supports [[tenant.token]])",
                           default="/tmp/sitewhere/segments", group="stor"),
                      Attr("rank", "Integer", "engine rank owning this store", default=0, group="stor"),
                      Attr("rotateBytes", "Integer", "segment file size before rotation", default=1 << 30,
                           group="stor"),
                      Attr("retentionBytes", "Integer", "bytes kept on disk (0 = unbounded)", default=0, group="stor"),
                      Attr("directIo", "Boolean", "O_DIRECT writes", default=True, group="perf")]))


class FilterProvider(ModelProvider):
    """Outbound connector filters (reference CommonConnectorRoles / OutboundConnectorsModelProvider filters)."""

    def initialize_roles(self):
        self.role(Role("connector-filters", "Filters", key="filters", multiple=True, reorderable=True))

    def initialize_elements(self):
        op = Attr("operation", "String", "include | exclude", default="include", choices=("include", "exclude"),
                  group="flt")
        self.element(Element("Area Filter", "connector-filters", ("area",), "Events of one area.", [
            Attr("areaToken", "String", "area token", required=True, group="flt"), op], icon="filter"))
        self.element(Element("Device Type Filter", "connector-filters", ("device-type",),
                             "Events of devices of one type.", [
                                 Attr("deviceTypeToken", "String", "device type token", required=True, group="flt"), op],
                             icon="filter"))
        self.element(Element("Event Type Filter", "connector-filters", ("event-type",), "Events of the listed types.", [
            Attr("eventTypes", "StringList", "Measurement | Location | Alert | CommandInvocation | ...",
                 required=True, group="flt")], icon="filter"))
        self.element(Element("Scripted Filter", "connector-filters", ("script",),
                             "filter(event, context) -> True skips the event.", [script_attr()], icon="code"))
