"""Microservice runtime: global and multitenant services, tenant engines, heartbeats, state.

Reference (``sitewhere-microservice``):
  * ``Microservice.java:182-237`` initialize (metrics, management API, state producer, topology,
    log producer), heartbeat every 20 s ``:86, 734-754``, wait for instance bootstrap ``:330-350``
  * ``configuration/ConfigurableMicroservice.java:208-448`` -- configuration monitor over
    ``/<instance>/conf``; restart chain Stop -> Terminate -> Initialize -> Start on change
  * ``multitenant/MultitenantMicroservice.java:54-572`` -- initialized / failed / initializing engine
    maps, tenant-init queue drained by a 5-thread pool, engines discovered from ``/conf/tenants``,
    ``assureTenantEngineAvailable`` gating RPCs, restart of an engine when its config changes
  * ``multitenant/MicroserviceTenantEngine.java`` + ``operations/*`` -- per-tenant configuration,
    Initialize (waits <= 60 s for the tenant bootstrap marker) -> Start -> Bootstrap under an
    inter-process mutex with a ``bootstrapped`` marker, state published on every change
  * ``MicroserviceApplication.java:48-205`` -- exit codes 2 (init/start failure) / 3 (unhandled)
  * ``logging/MicroserviceLogProducer.java`` -- every log line forwarded to ``instance-logging``
"""
from __future__ import annotations

import json
import logging
import os
import queue
import secrets
import socket
import threading
import time
import uuid

from ..bus import payloads
from ..bus.log import EventBus
from ..bus.naming import TopicNaming
from ..coord.store import NODE_ADDED, NODE_REMOVED, NODE_UPDATED, Coordination, InterProcessMutex, NodeExistsError
from ..core.errors import SiteWhereException, TenantEngineNotAvailableException
from ..core.lifecycle import (CompositeLifecycleStep, LifecycleComponent, LifecycleComponentType,
                              LifecycleProgressMonitor, LifecycleStatus, SimpleLifecycleStep,
                              TenantEngineLifecycleComponent)
from ..core.metrics import MetricRegistry, MetricsReporter
from ..core.security import SystemUser, TokenManagement, current_authentication
from ..core.trace_export import configure_tracing
from ..core.tracing import global_tracer
from ..models.domain import Tenant
from ..rpc.transport import GrpcChannel, LocalChannel, RpcServer, ServiceProxy, ServiceResolver
from .config import InstanceSettings, dump_document, parse_document, substitute
from .scripting import SCRIPT_TEMPLATES, ScriptManagement, ScriptRunner
from .topology import ApiDemux, NoLiveReplicaException, TopologyStateAggregator


# RPC service name -> owning microservice identifier (used to discover remote replicas).
SERVICE_OWNERS = {
    "DeviceManagement": "device-management", "DeviceEventManagement": "event-management",
    "AssetManagement": "asset-management", "BatchManagement": "batch-operations",
    "ScheduleManagement": "schedule-management", "TenantManagement": "tenant-management",
    "UserManagement": "user-management", "DeviceStateManagement": "device-state",
    "LabelGeneration": "label-generation", "StreamingMedia": "streaming-media", "EventSearch": "event-search",
    "EventSources": "event-sources", "InboundProcessing": "inbound-processing",
    "DeviceRegistration": "device-registration", "CommandDelivery": "command-delivery",
    "OutboundConnectors": "outbound-connectors", "RuleProcessing": "rule-processing",
}


def service_owner(service: str) -> str | None:
    if service.startswith(("MicroserviceManagement.", "MultitenantManagement.")):
        return service.split(".", 1)[1]
    return SERVICE_OWNERS.get(service)


class RoutingChannel:
    """Co-located services go through the in-process channel; everything else through an ApiDemux
    (topology-discovered gRPC replicas, round-robin, tenant-availability checks)."""

    def __init__(self, instance: "Instance"):
        self.instance = instance
        self.topology: TopologyStateAggregator | None = None
        self._demux: dict[str, ApiDemux] = {}
        self._lock = threading.Lock()

    def demux(self, identifier: str) -> ApiDemux:
        with self._lock:
            d = self._demux.get(identifier)
            if d is None:
                if self.topology is None:
                    raise SiteWhereException("no topology available for remote service discovery")
                jwt = self.instance.system_jwt()
                d = ApiDemux(identifier, self.topology, lambda addr: GrpcChannel(addr, jwt))
                self._demux[identifier] = d
            return d

    def call(self, service, method, *args, tenant=None, **kwargs):
        inst = self.instance
        if service in inst.resolver.names() or not inst.network_rpc:
            return inst.local_channel.call(service, method, *args, tenant=tenant, **kwargs)
        owner = service_owner(service)
        if owner is None:
            raise SiteWhereException(f"unknown service {service}")
        from ..rpc.transport import _tenant_for_call
        ch = self.demux(owner).get_channel(_tenant_for_call(tenant) if SERVICE_OWNERS.get(service) and
                                           service not in ("TenantManagement", "UserManagement") else None)
        return ch.call(service, method, *args, tenant=tenant, **kwargs)

    def proxy(self, service: str, tenant: str | None = None):
        return ServiceProxy(self, service, tenant)


class Instance:
    """Shared infrastructure of one SiteWhere instance as seen from this process."""

    def __init__(self, settings: InstanceSettings | None = None, bus: EventBus | None = None,
                 coord: Coordination | None = None, tokens: TokenManagement | None = None,
                 jwt_secret: str | None = None, network_rpc: bool = False):
        self.settings = settings or InstanceSettings.from_env()
        self.bus = bus or EventBus(None, default_partitions=8)
        self.coord = coord or Coordination()
        self.tokens = tokens or TokenManagement(jwt_secret or os.environ.get("SITEWHERE_JWT_SECRET")
                                                or self._shared_jwt_secret())
        self.naming = TopicNaming(self.settings.product_id, self.settings.instance_id)
        self.resolver = ServiceResolver()
        self.system_user = SystemUser(self.tokens)
        self.local_channel = LocalChannel(self.resolver, self.tokens, self.system_user.authentication().jwt,
                                          mode=self.settings.local_rpc)
        self.router = RoutingChannel(self)
        self.network_rpc = network_rpc
        self.microservices: dict[str, "Microservice"] = {}
        self.scripts = ScriptManagement(self.coord, self.path("scripts"))

    def _shared_jwt_secret(self) -> str:
        """One random HS512 secret per instance, created by whichever process gets there first and
        shared with every other process through the coordination store (the reference hard-codes
        "secret", ``TokenManagement.java:42-45``; a fixed default would let anyone who reads the source
        forge tokens).  Access to the coordination store is the trust boundary, as ZooKeeper is for
        the reference's configuration."""
        path = self.path("security", "jwt-secret")
        try:
            self.coord.create(path, secrets.token_hex(32).encode())
        except NodeExistsError:
            pass
        return self.coord.get(path)[0].decode()

    # coordination paths ---------------------------------------------------------
    def path(self, *parts) -> str:
        return "/" + "/".join([self.settings.product_id, self.settings.instance_id, *parts])

    def conf_path(self, *parts) -> str:
        return self.path("conf", *parts)

    def bootstrapped_marker(self) -> str:
        return self.path("state", "bootstrapped")

    def tenant_conf_path(self, tenant: str, *parts) -> str:
        return self.conf_path("tenants", tenant, *parts)

    def system_jwt(self) -> str:
        return self.system_user.authentication().jwt


class _WaitingChannel:
    """Retries calls that fail with TenantEngineNotAvailable (100 ms -> 3 s backoff, bounded)."""

    def __init__(self, channel, wait_s: float):
        self.ch, self.wait_s = channel, wait_s

    def call(self, service, method, *args, **kwargs):
        end = time.time() + self.wait_s
        delay = 0.1
        while True:
            try:
                return self.ch.call(service, method, *args, **kwargs)
            except (TenantEngineNotAvailableException, NoLiveReplicaException):
                if time.time() + delay > end:
                    raise
                time.sleep(delay)
                delay = min(3.0, delay * 2)


# ------------------------------------------------------------------------------ log forwarding
class BusLogHandler(logging.Handler):
    """Forwards log records to ``instance-logging`` through a queue + drain thread."""

    def __init__(self, bus: EventBus, topic: str, identifier: str, hostname: str, capacity: int = 10000):
        super().__init__(logging.INFO)
        self.bus, self.topic, self.identifier, self.hostname = bus, topic, identifier, hostname
        self.q: queue.Queue = queue.Queue(capacity)
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._drain, daemon=True, name="log-producer")
        self._t.start()

    def emit(self, record):
        try:
            m = {"microservice": self.identifier, "hostname": self.hostname, "level": record.levelname,
                 "logger": record.name, "message": record.getMessage(), "timestamp": int(record.created * 1000),
                 "tenant": getattr(record, "tenant", None)}
            if record.exc_info and record.exc_info[1] is not None:
                import traceback
                e = record.exc_info[1]
                m["exception"] = {"message": f"{type(e).__name__}: {e}", "frames": [
                    {"module": f.filename.rsplit("/", 1)[-1].removesuffix(".py"), "function": f.name,
                     "file": f.filename, "line": f.lineno} for f in traceback.extract_tb(record.exc_info[2])]}
            self.q.put_nowait(m)
        except queue.Full:
            pass

    def _drain(self):
        prod = self.bus.producer()
        while not self._stop.is_set():
            try:
                m = self.q.get(timeout=0.2)
            except queue.Empty:
                continue
            try:
                prod.send(self.topic, self.hostname, payloads.encode_log(m))
            except Exception:
                pass

    def close(self):
        self._stop.set()
        super().close()


# ------------------------------------------------------------------------------ management APIs
class MicroserviceManagementApi:
    """Per-process management API (reference microservice-management.proto, 7 RPCs)."""

    def __init__(self, ms: "Microservice"):
        self._ms = ms

    def get_configuration_model(self):
        m = self._ms.configuration_model()
        return m.to_dict() if m else None

    def get_global_configuration(self) -> dict:
        return self._ms.global_configuration()

    def _check(self, doc: dict, scope: str):
        """Reject a document the service's configuration model does not accept (the reference
        parses tenant XML against the service schema before applying it)."""
        m = self._ms.configuration_model()
        if m is not None and self._ms.multitenant == (scope == "tenant"):
            errs = m.validate(doc)
            if errs:
                raise SiteWhereException(f"invalid {self._ms.identifier} {scope} configuration: " + "; ".join(errs))

    def update_global_configuration(self, doc: dict) -> dict:
        self._check(doc, "global")
        self._ms.instance.coord.put(self._ms.config_path(), dump_document(doc))
        return doc

    def get_tenant_configuration(self, tenant: str) -> dict:
        return self._ms.tenant_configuration(tenant)

    def update_tenant_configuration(self, tenant: str, doc: dict) -> dict:
        self._check(doc, "tenant")
        self._ms.instance.coord.put(self._ms.tenant_config_path(tenant), dump_document(doc))
        return doc

    def get_script_templates(self) -> list:
        return sorted(SCRIPT_TEMPLATES.get(self._ms.identifier, {}))

    def get_script_template_content(self, template_id: str) -> str:
        return SCRIPT_TEMPLATES.get(self._ms.identifier, {}).get(template_id, "")

    def get_state(self) -> dict:
        return self._ms.state_tree()


class MultitenantManagementApi:
    def __init__(self, ms: "MultitenantMicroservice"):
        self._ms = ms

    def check_tenant_engine_available(self, tenant: str | None = None) -> bool:
        if tenant is None:                  # reference form: the tenant travels in the call metadata
            auth = current_authentication()
            tenant = auth.tenant if auth is not None else None
        e = self._ms.tenant_engines.get(tenant)
        return e is not None and e.status == LifecycleStatus.Started


# ------------------------------------------------------------------------------ microservice
class Microservice(LifecycleComponent):
    """Base microservice: identity, heartbeats, state reporting, topology, metrics, management API."""

    identifier = "microservice"
    name = "Microservice"
    component_type = LifecycleComponentType.Microservice
    multitenant = False

    def __init__(self, instance: Instance, hostname: str | None = None):
        super().__init__(self.name)
        self.instance = instance
        self.hostname = hostname or f"{self.identifier}-{socket.gethostname()}-{uuid.uuid4().hex[:6]}"
        self.microservice = self
        self.metrics = MetricRegistry()
        self.tracer = global_tracer()
        if instance.settings.tracer_server:
            configure_tracing(instance.settings.tracer_server, instance.settings.tracer_sample_rate,
                              instance.settings.product_id)
        self.producer = instance.bus.producer()
        self.topology = TopologyStateAggregator(instance.bus, instance.naming.microservice_state_updates(),
                                                self.hostname, instance.settings.topology_eviction_s)
        self.rpc_server: RpcServer | None = None
        self._hb_stop = threading.Event()
        self._hb: threading.Thread | None = None
        self._reporter: MetricsReporter | None = None
        self.log_handler: BusLogHandler | None = None
        self.scripts = ScriptRunner()
        if self.scripts.isolation == "process":
            # start the sandboxed worker now, before any tenant engine initialises a GPU in this
            # process (a process that has opened the GPU should not fork + exec children)
            self.scripts.sandbox().ensure_started()
        self.management = MicroserviceManagementApi(self)
        self.config: dict = {}
        self._demuxes: dict[str, ApiDemux] = {}
        self.add_status_listener(lambda c, o, n: self.publish_state())

    # ---- identity / state ---------------------------------------------------
    @property
    def api_address(self) -> str | None:
        return self.rpc_server.address if self.rpc_server and self.rpc_server.port else None

    def publish_state(self):
        msg = {"type": "microservice", "identifier": self.identifier, "hostname": self.hostname,
               "status": self.status.value, "apiAddress": self.api_address, "timestamp": int(time.time() * 1000)}
        try:
            self.producer.send(self.instance.naming.microservice_state_updates(), self.identifier,
                               json.dumps(msg).encode())
        except Exception:
            pass

    def publish_tenant_state(self, tenant: str, status: LifecycleStatus):
        msg = {"type": "tenant", "identifier": self.identifier, "hostname": self.hostname, "tenant": tenant,
               "status": status.value, "timestamp": int(time.time() * 1000)}
        self.producer.send(self.instance.naming.microservice_state_updates(), self.identifier, json.dumps(msg).encode())

    def _heartbeat(self):
        while not self._hb_stop.wait(self.instance.settings.heartbeat_s):
            self.publish_state()

    # ---- configuration ------------------------------------------------------
    def config_path(self) -> str:
        return self.instance.conf_path(f"{self.identifier}.json")

    def default_configuration(self) -> dict:
        return {}

    def global_configuration(self) -> dict:
        raw = self.instance.coord.get_data(self.config_path())
        doc = parse_document(raw) if raw else self.default_configuration()
        return substitute(doc, self.instance.settings.extra)

    def configuration_model(self):
        from ..configuration import model_for
        return model_for(self.identifier)

    def tenant_config_path(self, tenant: str) -> str:
        return self.instance.tenant_conf_path(tenant, f"{self.identifier}.json")

    def tenant_configuration(self, tenant: str) -> dict:
        raw = self.instance.coord.get_data(self.tenant_config_path(tenant))
        return parse_document(raw) if raw else {}

    # ---- service discovery ---------------------------------------------------
    def demux(self, identifier: str) -> ApiDemux:
        d = self._demuxes.get(identifier)
        if d is None:
            jwt = self.instance.system_jwt()
            factory = (lambda addr: GrpcChannel(addr, jwt)) if self.instance.network_rpc else (lambda addr: self.instance.local_channel)
            d = ApiDemux(identifier, self.topology, factory, local_channel=self.instance.local_channel)
            self._demuxes[identifier] = d
        return d

    def api(self, service: str, tenant: str | None = None, wait_s: float = 30.0):
        """Typed proxy to a service (co-located: in-process channel; remote: gRPC).  Calls made while
        the target tenant engine is still starting wait for it with backoff, like the reference's
        ``MultitenantApiDemux.waitForCorrespondingTenantEngineAvailable``."""
        return ServiceProxy(_WaitingChannel(self.instance.router, wait_s), service, tenant)

    # ---- hooks ----------------------------------------------------------------
    def register_services(self, resolver: ServiceResolver):
        """Register this service's RPC implementations."""

    def microservice_initialize(self, monitor):
        pass

    def microservice_start(self, monitor):
        pass

    def microservice_stop(self, monitor):
        pass

    def microservice_terminate(self, monitor):
        pass

    def configuration_updated(self, doc: dict):
        """Global configuration changed (default: restart configuration)."""
        self.restart_configuration()

    def restart_configuration(self):
        mon = LifecycleProgressMonitor(f"{self.identifier}-reconfigure")
        self.microservice_stop(mon)
        self.config = self.global_configuration()
        self.microservice_initialize(mon)
        self.microservice_start(mon)

    # ---- lifecycle --------------------------------------------------------------
    def wait_for_instance_initialization(self, timeout_s: float = 60.0):
        with self.tracer.start_span("Wait for instance bootstrap"):
            if not self.instance.coord.wait_for(self.instance.bootstrapped_marker(), timeout_s):
                raise SiteWhereException("instance was not bootstrapped in time")

    def requires_instance_bootstrap(self) -> bool:
        return True

    def initialize(self, monitor):
        inst = self.instance
        self.instance.microservices[self.hostname] = self
        steps = CompositeLifecycleStep(f"Initialize {self.name}")
        steps.add_step(SimpleLifecycleStep("Log producer", lambda m: self._init_logging()))
        steps.add_step(SimpleLifecycleStep("Coordination", lambda m: inst.coord.ensure(inst.conf_path())))
        steps.add_step(SimpleLifecycleStep("Register RPC services", lambda m: self._register_rpc()))
        steps.add_initialize_step(self, self.topology, require=True)
        if inst.router.topology is None:
            inst.router.topology = self.topology
        steps.execute(monitor)
        if inst.settings.log_metrics:
            self._reporter = MetricsReporter(self.metrics, lambda s: self.logger.info("metrics %s", s),
                                             inst.settings.metrics_period_s)
        if self.requires_instance_bootstrap():
            self.wait_for_instance_initialization()
        self.config = self.global_configuration()
        self.microservice_initialize(monitor)

    def _init_logging(self):
        self.log_handler = BusLogHandler(self.instance.bus, self.instance.naming.instance_logging(), self.identifier,
                                         self.hostname)
        logging.getLogger(f"sitewhere.{self.name}").addHandler(self.log_handler)

    def _register_rpc(self):
        res = self.instance.resolver
        self.register_services(res)
        res.add_global(f"MicroserviceManagement.{self.identifier}", self.management)
        if self.instance.network_rpc:
            st = self.instance.settings
            self.rpc_server = RpcServer(res, self.instance.tokens, port=st.grpc_port, host=st.grpc_host,
                                        advertise_host=st.grpc_advertise_host, identifier=self.identifier)

    def start(self, monitor):
        if self.rpc_server is not None:
            self.start_nested_component(self.rpc_server, monitor, require=True)
        self.start_nested_component(self.topology, monitor, require=True)
        self._hb_stop.clear()
        self._hb = threading.Thread(target=self._heartbeat, daemon=True, name=f"heartbeat-{self.identifier}")
        self._hb.start()
        if self._reporter:
            self._reporter.start()
        self._cancel_watch = self.instance.coord.watch_tree(self.config_path(), self._on_config_event, initial=False)
        self.microservice_start(monitor)

    def _on_config_event(self, kind, path, data):
        if kind in (NODE_UPDATED, NODE_ADDED) and path == self.config_path():
            try:
                self.configuration_updated(parse_document(data or b""))
            except Exception:
                self.logger.exception("configuration update failed")

    def stop(self, monitor):
        if getattr(self, "_cancel_watch", None):
            self._cancel_watch()
        self.microservice_stop(monitor)
        self._hb_stop.set()
        if self._reporter:
            self._reporter.stop()
        self.stop_nested_component(self.topology, monitor)
        if self.rpc_server is not None:
            self.stop_nested_component(self.rpc_server, monitor)

    def terminate(self, monitor):
        self.microservice_terminate(monitor)
        self.scripts.close()
        if self.log_handler:
            self.log_handler.close()
        self.instance.microservices.pop(self.hostname, None)


class GlobalMicroservice(Microservice):
    """Single-configuration service (instance, tenant, user management, web-rest)."""


_SCRIPT_ID = __import__("re").compile(r"^[A-Za-z0-9_.\-]+$")


class MicroserviceTenantEngine(TenantEngineLifecycleComponent):
    """Per-tenant engine of a multitenant microservice."""

    component_type = LifecycleComponentType.TenantEngine

    def __init__(self, microservice: "MultitenantMicroservice", tenant: Tenant):
        super().__init__(f"{microservice.identifier}:{tenant.token}")
        self.tenant_engine = self
        self.ms = microservice
        self.microservice = microservice
        self.tenant = tenant
        self.config: dict = {}
        self.api = None  # RPC implementation for this tenant

    def script_source(self, ref) -> str:
        """Source of a configured script.  ``{"scriptId": id[, "version": v]}`` or a bare script id
        names a versioned script in script management (tenant scope, then global, of this
        microservice; the active version unless pinned) -- the reference's ``scriptId`` attributes
        (``ZookeeperScriptManagement``); anything else is inline source."""
        from ..core.errors import NotFoundException
        sid, ver = (ref.get("scriptId") or ref.get("id"), ref.get("version")) if isinstance(ref, dict) else (ref, None)
        if isinstance(sid, str) and _SCRIPT_ID.match(sid):
            for scope in (self.tenant.token, "global"):
                try:
                    return self.ms.instance.scripts.get_content(scope, self.ms.identifier, sid, ver)
                except NotFoundException:
                    continue
            raise SiteWhereException(f"script {sid!r} not found for {self.ms.identifier} "
                                     f"(tenant {self.tenant.token} or global scope)")
        if isinstance(ref, dict):
            raise SiteWhereException(f"invalid script reference {ref!r}")
        return ref

    # hooks ----------------------------------------------------------------------
    def tenant_initialize(self, monitor):
        pass

    def tenant_start(self, monitor):
        pass

    def tenant_stop(self, monitor):
        pass

    def tenant_bootstrap(self, dataset_template: str, monitor):
        pass

    # lifecycle --------------------------------------------------------------------
    def load_configuration(self) -> dict:
        doc = self.ms.tenant_configuration(self.tenant.token)
        return substitute(doc, self.ms.instance.settings.extra, {"tenant.id": self.tenant.id,
                                                                  "tenant.token": self.tenant.token,
                                                                  "id": self.tenant.id, "token": self.tenant.token})

    def initialize(self, monitor):
        self.config = self.load_configuration()
        self.tenant_initialize(monitor)

    def start(self, monitor):
        self.tenant_start(monitor)

    def stop(self, monitor):
        self.tenant_stop(monitor)

    def lifecycle_status_changed(self, old, new):
        try:
            self.ms.publish_tenant_state(self.tenant.token, new)
        except Exception:
            pass

    def bootstrap(self, monitor=None):
        """Run the dataset bootstrap once per (tenant, microservice) across all replicas."""
        inst = self.ms.instance
        marker = inst.tenant_conf_path(self.tenant.token, self.ms.identifier, "bootstrapped")
        if inst.coord.exists(marker):
            return False
        with self.ms.tracer.start_span(f"Bootstrap {self.component_name}"):
            with InterProcessMutex(inst.coord, inst.tenant_conf_path(self.tenant.token, self.ms.identifier, "lock")):
                if inst.coord.exists(marker):
                    return False
                self.tenant_bootstrap(self.tenant.dataset_template_id, monitor or LifecycleProgressMonitor())
                inst.coord.ensure(marker)
                return True


class MultitenantMicroservice(Microservice):
    multitenant = True
    tenant_wait_s = 60.0

    def __init__(self, instance: Instance, hostname: str | None = None):
        super().__init__(instance, hostname)
        self.tenant_engines: dict[str, MicroserviceTenantEngine] = {}
        self.failed_tenant_engines: dict[str, MicroserviceTenantEngine] = {}
        self.initializing: set[str] = set()
        self._q: queue.Queue = queue.Queue()
        self._workers: list[threading.Thread] = []
        self._tlock = threading.RLock()
        self._stop_workers = threading.Event()
        self.mt_management = MultitenantManagementApi(self)

    # hooks ------------------------------------------------------------------------
    def create_tenant_engine(self, tenant: Tenant) -> MicroserviceTenantEngine:
        raise NotImplementedError

    def service_names(self) -> list[str]:
        """RPC service names resolved per tenant engine (engine.api)."""
        return []

    def register_services(self, resolver):
        for name in self.service_names():
            resolver.add_tenant(name, self._engine_api(name))
        resolver.add_global(f"MultitenantManagement.{self.identifier}", self.mt_management)
        resolver.add_global("MultitenantManagement", self.mt_management)

    def _engine_api(self, name):
        def resolve(tenant: str):
            e = self.assure_tenant_engine_available(tenant)
            api = e.api
            if isinstance(api, dict):
                return api[name]
            return api
        return resolve

    # tenant engines -------------------------------------------------------------
    def get_tenant_engine(self, tenant: str) -> MicroserviceTenantEngine | None:
        return self.tenant_engines.get(tenant)

    def assure_tenant_engine_available(self, tenant: str) -> MicroserviceTenantEngine:
        e = self.tenant_engines.get(tenant)
        if e is None or e.status not in (LifecycleStatus.Started, LifecycleStatus.StartedWithErrors):
            raise TenantEngineNotAvailableException(f"{self.identifier}: tenant engine {tenant} not available")
        return e

    def wait_for_tenant_engine(self, tenant: str, timeout_s: float = 30.0) -> MicroserviceTenantEngine:
        end = time.time() + timeout_s
        while time.time() < end:
            e = self.tenant_engines.get(tenant)
            if e is not None and e.status in (LifecycleStatus.Started, LifecycleStatus.StartedWithErrors):
                return e
            if tenant in self.failed_tenant_engines:
                raise SiteWhereException(f"tenant engine {tenant} failed: "
                                         f"{self.failed_tenant_engines[tenant].lifecycle_error}")
            time.sleep(0.02)
        raise TenantEngineNotAvailableException(f"tenant engine {tenant} did not start")

    def lookup_tenant(self, token: str) -> Tenant:
        return self.api("TenantManagement").get_tenant_by_token(token)

    def _worker(self):
        while not self._stop_workers.is_set():
            try:
                token = self._q.get(timeout=0.2)
            except queue.Empty:
                continue
            try:
                self._start_tenant_engine(token)
            except Exception:
                self.logger.exception("tenant engine %s failed to start", token)
            finally:
                with self._tlock:
                    self.initializing.discard(token)

    def _start_tenant_engine(self, token: str):
        inst = self.instance
        sysuser = inst.system_user
        tenant = sysuser.run(self.lookup_tenant, None, token)
        if tenant is None:
            return
        # InitializeTenantEngineOperation: wait for the tenant configuration bootstrap marker
        if not inst.coord.wait_for(inst.tenant_conf_path(token, "bootstrapped"), self.tenant_wait_s):
            raise SiteWhereException(f"tenant {token} configuration not bootstrapped")
        engine = self.create_tenant_engine(tenant)
        engine.microservice = self
        mon = LifecycleProgressMonitor(f"{self.identifier}:{token}")
        with self.tracer.start_span(f"Initialize tenant engine {token}"):
            sysuser.run(lambda: self.initialize_nested_component(engine, mon, False), token)
        if engine.status == LifecycleStatus.InitializationError:
            self.failed_tenant_engines[token] = engine
            return
        sysuser.run(lambda: engine.lifecycle_start(mon), token)
        if engine.status == LifecycleStatus.LifecycleError:
            self.failed_tenant_engines[token] = engine
            return
        self._register(engine)
        with self._tlock:
            self.tenant_engines[token] = engine
            self.failed_tenant_engines.pop(token, None)
        sysuser.run(engine.bootstrap, token, mon)

    def add_tenant(self, token: str):
        with self._tlock:
            if token in self.tenant_engines or token in self.initializing:
                return
            self.initializing.add(token)
        self._q.put(token)

    def remove_tenant_engine(self, token: str):
        with self._tlock:
            e = self.tenant_engines.pop(token, None)
            self.failed_tenant_engines.pop(token, None)
        if e is not None:
            mon = LifecycleProgressMonitor()
            e.lifecycle_stop(mon)
            e.lifecycle_terminate(mon)
            self.remove_nested_component(e)

    def restart_tenant_engine(self, token: str):
        """MultitenantMicroservice.restartTenantEngine: stop + terminate + re-enqueue."""
        self.remove_tenant_engine(token)
        self.add_tenant(token)

    def _on_tenants_event(self, kind, path, data):
        inst = self.instance
        base = inst.conf_path("tenants")
        rel = path[len(base):].strip("/").split("/")
        if not rel or not rel[0]:
            return
        token = rel[0]
        if kind == NODE_ADDED and len(rel) == 2 and rel[1] == "bootstrapped":
            self.add_tenant(token)
        elif kind == NODE_UPDATED and len(rel) == 2 and rel[1] == f"{self.identifier}.json":
            if token in self.tenant_engines:
                self.restart_tenant_engine(token)
        elif kind == NODE_REMOVED and len(rel) == 1:
            self.remove_tenant_engine(token)

    def microservice_start_tenants(self):
        inst = self.instance
        inst.coord.ensure(inst.conf_path("tenants"))
        for token in inst.coord.children(inst.conf_path("tenants")):
            if inst.coord.exists(inst.tenant_conf_path(token, "bootstrapped")):
                self.add_tenant(token)

    def start(self, monitor):
        super().start(monitor)
        self._stop_workers.clear()
        self._workers = [threading.Thread(target=self._worker, daemon=True, name=f"tenant-ops-{i}")
                         for i in range(self.instance.settings.tenant_ops_threads)]
        for w in self._workers:
            w.start()
        self._cancel_tenant_watch = self.instance.coord.watch_tree(self.instance.conf_path("tenants"),
                                                                   self._on_tenants_event, initial=False)
        self.microservice_start_tenants()

    def configuration_updated(self, doc: dict):
        """Global configuration change restarts configuration and every tenant engine (reference :381-409)."""
        super().configuration_updated(doc)
        for t in list(self.tenant_engines):
            self.restart_tenant_engine(t)

    def stop(self, monitor):
        if getattr(self, "_cancel_tenant_watch", None):
            self._cancel_tenant_watch()
        for t in list(self.tenant_engines):
            self.remove_tenant_engine(t)
        self._stop_workers.set()
        for w in self._workers:
            w.join(timeout=2)
        super().stop(monitor)

    def state_tree(self) -> dict:
        d = super().state_tree()
        d["tenantEngines"] = {t: e.status.value for t, e in self.tenant_engines.items()}
        d["failedTenantEngines"] = {t: str(e.lifecycle_error) for t, e in self.failed_tenant_engines.items()}
        return d


def run_microservice(ms: Microservice, monitor: LifecycleProgressMonitor | None = None) -> int:
    """MicroserviceApplication: initialize + start; returns the process exit code (0 / 2)."""
    mon = monitor or LifecycleProgressMonitor(ms.identifier)
    with ms.tracer.start_span(f"Start microservice {ms.identifier}"):
        ms.lifecycle_initialize(mon)
        if ms.status == LifecycleStatus.InitializationError:
            ms.logger.error("initialization failed: %s", ms.lifecycle_error)
            return 2
        ms.lifecycle_start(mon)
        if ms.status == LifecycleStatus.LifecycleError:
            ms.logger.error("start failed: %s", ms.lifecycle_error)
            return 2
    return 0


def shutdown_microservice(ms: Microservice):
    mon = LifecycleProgressMonitor(ms.identifier)
    ms.lifecycle_stop(mon)
    ms.lifecycle_terminate(mon)
