"""Topic naming (reference: ``sitewhere-microservice/.../kafka/KafkaTopicNaming.java:21-219``).

``<product>.<instance>.global.<suffix>`` and ``<product>.<instance>.tenant.<tenantId>.<suffix>``.
"""
from __future__ import annotations

SEP = "."
GLOBAL = "global"
TENANT = "tenant"

# global suffixes
MICROSERVICE_STATE_UPDATES = "microservice-state-updates"
INSTANCE_TOPOLOGY_UPDATES = "instance-topology-updates"
TENANT_MODEL_UPDATES = "tenant-model-updates"
INSTANCE_LOGGING = "instance-logging"
# tenant suffixes
EVENT_SOURCE_DECODED_EVENTS = "event-source-decoded-events"
EVENT_SOURCE_FAILED_DECODE_EVENTS = "event-source-failed-decode-events"
INBOUND_REPROCESS_EVENTS = "inbound-reprocess-events"
INBOUND_PERSISTED_EVENTS = "inbound-persisted-events"
INBOUND_DEVICE_REGISTRATION_EVENTS = "inbound-device-registration-events"
INBOUND_UNREGISTERED_DEVICE_EVENTS = "inbound-unregistered-device-events"
INBOUND_ENRICHED_EVENTS = "inbound-enriched-events"
INBOUND_ENRICHED_COMMAND_INVOCATIONS = "inbound-enriched-command-invocations"
UNDELIVERED_COMMAND_INVOCATIONS = "undelivered-command-invocations"

GLOBAL_SUFFIXES = [MICROSERVICE_STATE_UPDATES, INSTANCE_TOPOLOGY_UPDATES, TENANT_MODEL_UPDATES, INSTANCE_LOGGING]
TENANT_SUFFIXES = [EVENT_SOURCE_DECODED_EVENTS, EVENT_SOURCE_FAILED_DECODE_EVENTS, INBOUND_REPROCESS_EVENTS,
                   INBOUND_PERSISTED_EVENTS, INBOUND_DEVICE_REGISTRATION_EVENTS, INBOUND_UNREGISTERED_DEVICE_EVENTS,
                   INBOUND_ENRICHED_EVENTS, INBOUND_ENRICHED_COMMAND_INVOCATIONS, UNDELIVERED_COMMAND_INVOCATIONS]


class TopicNaming:
    def __init__(self, product: str = "sitewhere", instance: str = "sitewhere1"):
        self.product = product
        self.instance = instance

    def prefix(self) -> str:
        return f"{self.product}{SEP}{self.instance}"

    def global_prefix(self) -> str:
        return f"{self.prefix()}{SEP}{GLOBAL}{SEP}"

    def tenant_prefix(self, tenant_id: str) -> str:
        return f"{self.prefix()}{SEP}{TENANT}{SEP}{tenant_id}{SEP}"

    # global topics
    def microservice_state_updates(self) -> str:
        return self.global_prefix() + MICROSERVICE_STATE_UPDATES

    def instance_topology_updates(self) -> str:
        return self.global_prefix() + INSTANCE_TOPOLOGY_UPDATES

    def tenant_model_updates(self) -> str:
        return self.global_prefix() + TENANT_MODEL_UPDATES

    def instance_logging(self) -> str:
        return self.global_prefix() + INSTANCE_LOGGING

    # tenant topics
    def decoded_events(self, t: str) -> str:
        return self.tenant_prefix(t) + EVENT_SOURCE_DECODED_EVENTS

    def failed_decode_events(self, t: str) -> str:
        return self.tenant_prefix(t) + EVENT_SOURCE_FAILED_DECODE_EVENTS

    def inbound_reprocess_events(self, t: str) -> str:
        return self.tenant_prefix(t) + INBOUND_REPROCESS_EVENTS

    def inbound_persisted_events(self, t: str) -> str:
        return self.tenant_prefix(t) + INBOUND_PERSISTED_EVENTS

    def device_registration_events(self, t: str) -> str:
        return self.tenant_prefix(t) + INBOUND_DEVICE_REGISTRATION_EVENTS

    def unregistered_device_events(self, t: str) -> str:
        return self.tenant_prefix(t) + INBOUND_UNREGISTERED_DEVICE_EVENTS

    def inbound_enriched_events(self, t: str) -> str:
        return self.tenant_prefix(t) + INBOUND_ENRICHED_EVENTS

    def enriched_command_invocations(self, t: str) -> str:
        return self.tenant_prefix(t) + INBOUND_ENRICHED_COMMAND_INVOCATIONS

    def undelivered_command_invocations(self, t: str) -> str:
        return self.tenant_prefix(t) + UNDELIVERED_COMMAND_INVOCATIONS

    def all_tenant_topics(self, t: str) -> list[str]:
        return [self.tenant_prefix(t) + s for s in TENANT_SUFFIXES]

    def all_global_topics(self) -> list[str]:
        return [self.global_prefix() + s for s in GLOBAL_SUFFIXES]
