"""Assemble a whole SiteWhere instance -- every microservice -- in one process.

The reference deploys 19 microservices as separate JVMs behind Kafka/ZooKeeper/gRPC
(``deploy/``, Helm charts).  Here every microservice is the same lifecycle component whether it
runs alone (``python -m sitewhere_amd.serve <service>``) or co-located: this module is the
co-located form used by the tests, the demo server and the single-node deployment (one process per
node, the GPU inbound engine on that node's MI355X).  Start order follows the reference's
dependency waits: instance management first (it writes the bootstrap marker), then the global
services (users, tenants), then every multitenant service (each waits for tenant bootstrap markers).
"""
from __future__ import annotations

import os

import time

from .runtime.config import InstanceSettings
from .runtime.microservice import Instance, run_microservice, shutdown_microservice
from .services.asset_management import AssetManagementMicroservice
from .services.batch_operations import BatchOperationsMicroservice
from .services.command_delivery import CommandDeliveryMicroservice
from .services.device_management import DeviceManagementMicroservice
from .services.device_registration import DeviceRegistrationMicroservice
from .services.device_state import DeviceStateMicroservice
from .services.event_management import EventManagementMicroservice
from .services.event_sources import EventSourcesMicroservice
from .services.inbound_processing import InboundProcessingMicroservice
from .services.instance_management import InstanceManagementMicroservice
from .services.labels_media_search import (EventSearchMicroservice, LabelGenerationMicroservice,
                                           StreamingMediaMicroservice)
from .services.outbound_connectors import OutboundConnectorsMicroservice
from .services.rule_processing import RuleProcessingMicroservice
from .services.schedule_management import ScheduleManagementMicroservice
from .services.tenant_management import TenantManagementMicroservice
from .services.user_management import UserManagementMicroservice
from .web.rest import WebRestMicroservice

GLOBAL_SERVICES = [UserManagementMicroservice, TenantManagementMicroservice]
MULTITENANT_SERVICES = [
    DeviceManagementMicroservice, EventManagementMicroservice, AssetManagementMicroservice,
    EventSourcesMicroservice, InboundProcessingMicroservice, DeviceRegistrationMicroservice,
    DeviceStateMicroservice, RuleProcessingMicroservice, OutboundConnectorsMicroservice,
    CommandDeliveryMicroservice, BatchOperationsMicroservice, ScheduleManagementMicroservice,
    LabelGenerationMicroservice, StreamingMediaMicroservice, EventSearchMicroservice,
]
SERVICES_BY_ID = {c.identifier: c for c in [InstanceManagementMicroservice, *GLOBAL_SERVICES, *MULTITENANT_SERVICES,
                                            WebRestMicroservice]}


class SiteWhereInstance:
    """All microservices of one instance sharing the in-process bus, coordination store and RPC resolver."""

    def __init__(self, settings: InstanceSettings | None = None, template: str = "default",
                 services: list[str] | None = None, instance: Instance | None = None, rest_port: int = 0,
                 **instance_kw):
        self.instance = instance or Instance(settings or InstanceSettings.from_env(heartbeat_s=5.0), **instance_kw)
        self.template = template
        wanted = set(services) if services else None
        self.instance_management = InstanceManagementMicroservice(self.instance, template=template)
        self.services = [c(self.instance) for c in GLOBAL_SERVICES + MULTITENANT_SERVICES
                         if wanted is None or c.identifier in wanted]
        if wanted is None or "web-rest" in wanted:
            self.services.append(WebRestMicroservice(self.instance, port=rest_port))
        self.started = False

    def __getitem__(self, identifier: str):
        for s in [self.instance_management, *self.services]:
            if s.identifier == identifier:
                return s
        raise KeyError(identifier)

    def start(self, timeout_s: float = 60.0):
        # every microservice of the instance shares this interpreter: with the default 5 ms switch
        # interval a thread coming back from a native call (an engine submit, a store lookup) waits
        # up to 5 ms for a busy peer to yield.  The engine loops make many short native calls.
        import sys
        us = float(os.environ.get("SW_SWITCH_INTERVAL_US", "200"))
        if us > 0:
            sys.setswitchinterval(us / 1e6)
        if run_microservice(self.instance_management) != 0:
            raise RuntimeError(f"instance management failed: {self.instance_management.lifecycle_error}")
        for s in self.services:
            if run_microservice(s) != 0:
                raise RuntimeError(f"{s.identifier} failed: {s.lifecycle_error}")
        self.started = True
        self.instance_management.model_initialized.wait(timeout_s)
        return self

    def api(self, service: str, tenant: str | None = None):
        return self.instance.local_channel.proxy(service, tenant)

    def wait_for_tenant(self, token: str = "default", timeout_s: float = 60.0):
        """Block until every multitenant service has a started engine for ``token`` (and bootstrap ran)."""
        end = time.time() + timeout_s
        for s in self.services:
            if getattr(s, "multitenant", False):
                e = s.wait_for_tenant_engine(token, max(0.1, end - time.time()))
                bm = self.instance.tenant_conf_path(token, s.identifier, "bootstrapped")
                while not self.instance.coord.exists(bm) and time.time() < end:
                    time.sleep(0.02)
                _ = e
        return self

    @property
    def rest_app(self):
        return self["web-rest"].app

    def tenant_engine(self, identifier: str, token: str = "default"):
        return self[identifier].get_tenant_engine(token)

    def stop(self):
        for s in reversed(self.services):
            try:
                shutdown_microservice(s)
            except Exception:
                pass
        shutdown_microservice(self.instance_management)
        self.instance.bus.close()
        self.started = False

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()
