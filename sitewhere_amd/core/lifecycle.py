"""Lifecycle kernel: component state machine, nested components, composite steps, progress.

Reference: ``sitewhere-core-lifecycle`` --
  * ``LifecycleStatus.java:15-55`` (13 states)
  * ``LifecycleComponent.java:156-189`` initialize, ``:242-289`` start, ``:339-355`` pause,
    ``:397-445`` stop, ``:504+`` terminate; nested required/optional children ``:218-232, 319-329``;
    error aggregation into StartedWithErrors / StoppedWithErrors ``:262-268, 417-424``
  * ``CompositeLifecycleStep.java:72-97``, ``LifecycleProgressMonitor.java:94-100``
  * ``parameters/LifecycleComponentParameter.java`` (required parameter validation ``:138-146``)

Differences by design: the child registry is lock-protected (the reference uses a plain HashMap
mutated from tenant-op threads), and every transition opens a tracer span.
"""
from __future__ import annotations

import enum
import logging
import threading
import time
import uuid
from dataclasses import dataclass
from typing import Any, Callable

from .errors import ServerStartupException, SiteWhereException
from .tracing import Span, global_tracer


class LifecycleStatus(str, enum.Enum):
    Initializing = "Initializing"
    InitializationError = "InitializationError"
    Stopped = "Stopped"
    StoppedWithErrors = "StoppedWithErrors"
    Starting = "Starting"
    Started = "Started"
    StartedWithErrors = "StartedWithErrors"
    Pausing = "Pausing"
    Paused = "Paused"
    Stopping = "Stopping"
    Terminating = "Terminating"
    Terminated = "Terminated"
    LifecycleError = "LifecycleError"


class LifecycleComponentType(str, enum.Enum):
    """Coarse component classification (reference ``LifecycleComponentType``)."""
    Microservice = "Microservice"
    TenantEngine = "TenantEngine"
    DataStore = "DataStore"
    CacheProvider = "CacheProvider"
    InboundEventSource = "InboundEventSource"
    InboundEventReceiver = "InboundEventReceiver"
    DeviceEventDecoder = "DeviceEventDecoder"
    OutboundConnector = "OutboundConnector"
    RuleProcessor = "RuleProcessor"
    CommandDestination = "CommandDestination"
    CommandRouter = "CommandRouter"
    RegistrationManager = "RegistrationManager"
    BatchOperationManager = "BatchOperationManager"
    ScheduleManager = "ScheduleManager"
    SearchProvider = "SearchProvider"
    LabelGenerator = "LabelGenerator"
    Other = "Other"


# ------------------------------------------------------------------------------ progress
@dataclass
class LifecycleProgressContext:
    total_operations: int
    operation_name: str
    current: int = 0
    current_name: str = ""


class LifecycleProgressMonitor:
    """Stack of (opCount, name) contexts; reports progress and opens tracer spans."""

    def __init__(self, name: str = "lifecycle", listener: Callable[[dict], None] | None = None, tracer=None):
        self.name = name
        self.stack: list[LifecycleProgressContext] = []
        self.listener = listener
        self.tracer = tracer or global_tracer()
        self.messages: list[dict] = []

    def push_context(self, ctx: LifecycleProgressContext):
        self.stack.append(ctx)

    def pop_context(self):
        if self.stack:
            self.stack.pop()

    def start_progress(self, name: str):
        if self.stack:
            c = self.stack[-1]
            c.current += 1
            c.current_name = name
        self._report(name)

    def finish_progress(self):
        pass

    def _report(self, name: str):
        msg = {"monitor": self.name, "task": name, "level": len(self.stack),
               "progress": [(c.current, c.total_operations, c.operation_name) for c in self.stack]}
        self.messages.append(msg)
        if self.listener:
            self.listener(msg)

    def create_tracer_span(self, name: str) -> Span:
        return self.tracer.start_span(name)

    @staticmethod
    def handle_error_in_span(span: Span | None, exc: BaseException):
        if span is not None:
            span.set_error(exc)

    @staticmethod
    def finish_span(span: Span | None):
        if span is not None:
            span.finish()


# ------------------------------------------------------------------------------ parameters
@dataclass
class LifecycleComponentParameter:
    name: str
    value: Any = None
    required: bool = False
    default: Any = None


# ------------------------------------------------------------------------------ component
class LifecycleComponent:
    """Base class of every managed component.

    Subclasses override ``initialize/start/pause/stop/terminate`` hooks (all receive the
    progress monitor); the ``lifecycle_*`` wrappers handle state, errors, children and spans.
    """

    component_type = LifecycleComponentType.Other

    def __init__(self, name: str | None = None):
        self.component_id = uuid.uuid4()
        self.component_name = name or type(self).__name__
        self._status = LifecycleStatus.Stopped
        self.lifecycle_error: BaseException | None = None
        self._children: dict[uuid.UUID, LifecycleComponent] = {}
        self._children_lock = threading.RLock()
        self._listeners: list[Callable[[LifecycleComponent, LifecycleStatus, LifecycleStatus], None]] = []
        self.parameters: list[LifecycleComponentParameter] = []
        self.microservice = None
        self.logger = logging.getLogger(f"sitewhere.{self.component_name}")
        self.created = time.time()

    # ---- status -------------------------------------------------------------
    @property
    def status(self) -> LifecycleStatus:
        return self._status

    def set_status(self, s: LifecycleStatus):
        old = self._status
        self._status = s
        if old != s:
            for cb in list(self._listeners):
                try:
                    cb(self, old, s)
                except Exception:  # listeners never break the FSM
                    self.logger.exception("lifecycle listener failed")
            self.lifecycle_status_changed(old, s)

    def lifecycle_status_changed(self, old: LifecycleStatus, new: LifecycleStatus):
        """Hook (reference: MicroserviceTenantEngine publishes state on every change)."""

    def add_status_listener(self, cb):
        self._listeners.append(cb)

    @property
    def children(self) -> dict:
        with self._children_lock:
            return dict(self._children)

    # ---- parameters ---------------------------------------------------------
    def initialize_parameters(self):
        for p in self.parameters:
            if p.value is None:
                p.value = p.default

    def validate_parameters(self):
        for p in self.parameters:
            if p.required and p.value is None:
                raise SiteWhereException(
                    f"No value provided for required parameter '{p.name}'. Unable to initialize component.")

    # ---- hooks (override) ---------------------------------------------------
    def can_initialize(self) -> bool:
        return True

    def initialize(self, monitor: LifecycleProgressMonitor):
        pass

    def can_start(self) -> bool:
        return True

    def start(self, monitor: LifecycleProgressMonitor):
        pass

    def can_pause(self) -> bool:
        return False

    def pause(self, monitor: LifecycleProgressMonitor):
        pass

    def can_stop(self) -> bool:
        return True

    def stop(self, monitor: LifecycleProgressMonitor):
        pass

    def terminate(self, monitor: LifecycleProgressMonitor):
        pass

    # ---- wrappers -----------------------------------------------------------
    def _fail(self, span, exc: BaseException, status: LifecycleStatus):
        self.lifecycle_error = exc if isinstance(exc, SiteWhereException) else SiteWhereException(str(exc))
        self.lifecycle_error.__cause__ = exc
        self.set_status(status)
        self.logger.error("%s state transitioned to ERROR: %s", self.component_name, exc)
        LifecycleProgressMonitor.handle_error_in_span(span, exc)

    def lifecycle_initialize(self, monitor: LifecycleProgressMonitor | None = None):
        monitor = monitor or LifecycleProgressMonitor()
        span = monitor.create_tracer_span(f"Initialize {self.component_name}")
        try:
            self.initialize_parameters()
            self.validate_parameters()
            if not self.can_initialize():
                return
            self.lifecycle_error = None
            self.set_status(LifecycleStatus.Initializing)
            self.initialize(monitor)
            self.set_status(LifecycleStatus.Stopped)
        except BaseException as e:  # noqa: BLE001 -- mirrors reference catch(Throwable)
            self._fail(span, e, LifecycleStatus.InitializationError)
        finally:
            LifecycleProgressMonitor.finish_span(span)

    def _aggregate(self, ok: LifecycleStatus, bad: LifecycleStatus, bad_children) -> LifecycleStatus:
        for c in self.children.values():
            if c.status in bad_children:
                return bad
        return ok

    def lifecycle_start(self, monitor: LifecycleProgressMonitor | None = None):
        monitor = monitor or LifecycleProgressMonitor()
        span = monitor.create_tracer_span(f"Start {self.component_name}")
        try:
            if not self.can_start():
                return
            old = self.status
            self.set_status(LifecycleStatus.Starting)
            if old != LifecycleStatus.Paused:
                self.start(monitor)
            self.set_status(self._aggregate(LifecycleStatus.Started, LifecycleStatus.StartedWithErrors,
                                            (LifecycleStatus.LifecycleError, LifecycleStatus.StartedWithErrors)))
        except BaseException as e:  # noqa: BLE001
            self._fail(span, e, LifecycleStatus.LifecycleError)
        finally:
            LifecycleProgressMonitor.finish_span(span)

    def lifecycle_pause(self, monitor: LifecycleProgressMonitor | None = None):
        monitor = monitor or LifecycleProgressMonitor()
        self.set_status(LifecycleStatus.Pausing)
        try:
            self.pause(monitor)
            self.set_status(LifecycleStatus.Paused)
        except BaseException as e:  # noqa: BLE001
            self._fail(None, e, LifecycleStatus.LifecycleError)

    def lifecycle_stop(self, monitor: LifecycleProgressMonitor | None = None, constraints=None):
        monitor = monitor or LifecycleProgressMonitor()
        span = monitor.create_tracer_span(f"Stop {self.component_name}")
        try:
            if not self.can_stop():
                return
            self.set_status(LifecycleStatus.Stopping)
            self.stop(monitor)
            self.set_status(self._aggregate(LifecycleStatus.Stopped, LifecycleStatus.StoppedWithErrors,
                                            (LifecycleStatus.LifecycleError, LifecycleStatus.StoppedWithErrors)))
        except BaseException as e:  # noqa: BLE001
            self._fail(span, e, LifecycleStatus.LifecycleError)
        finally:
            LifecycleProgressMonitor.finish_span(span)

    def lifecycle_terminate(self, monitor: LifecycleProgressMonitor | None = None):
        monitor = monitor or LifecycleProgressMonitor()
        span = monitor.create_tracer_span(f"Terminate {self.component_name}")
        try:
            self.set_status(LifecycleStatus.Terminating)
            for c in list(self.children.values()):
                c.lifecycle_terminate(monitor)
            self.terminate(monitor)
            self.set_status(LifecycleStatus.Terminated)
        except BaseException as e:  # noqa: BLE001
            self._fail(span, e, LifecycleStatus.LifecycleError)
        finally:
            LifecycleProgressMonitor.finish_span(span)

    # ---- nested components --------------------------------------------------
    def _register(self, c: "LifecycleComponent"):
        with self._children_lock:
            self._children[c.component_id] = c

    def initialize_nested_component(self, c: "LifecycleComponent", monitor, require: bool = False):
        c.microservice = self.microservice
        c.lifecycle_initialize(monitor)
        if require and c.status == LifecycleStatus.InitializationError:
            raise ServerStartupException(c, f"Error initializing '{c.component_name}'", c.lifecycle_error)
        self._register(c)

    def start_nested_component(self, c: "LifecycleComponent", monitor, require: bool = False):
        c.lifecycle_start(monitor)
        if require and c.status == LifecycleStatus.LifecycleError:
            raise ServerStartupException(c, f"Unable to start '{c.component_name}'", c.lifecycle_error)
        self._register(c)

    def stop_nested_component(self, c: "LifecycleComponent", monitor):
        c.lifecycle_stop(monitor)

    def remove_nested_component(self, c: "LifecycleComponent"):
        with self._children_lock:
            self._children.pop(c.component_id, None)

    # ---- introspection --------------------------------------------------------
    def state_tree(self) -> dict:
        """Recursive status snapshot (reference ILifecycleComponentState for the admin UI)."""
        return {
            "componentId": str(self.component_id), "name": self.component_name,
            "type": self.component_type.value, "status": self.status.value,
            "error": str(self.lifecycle_error) if self.lifecycle_error else None,
            "children": [c.state_tree() for c in self.children.values()],
        }

    def find_components_of_type(self, t: LifecycleComponentType) -> list:
        out = [self] if self.component_type == t else []
        for c in self.children.values():
            out.extend(c.find_components_of_type(t))
        return out


class TenantEngineLifecycleComponent(LifecycleComponent):
    """Component scoped to a tenant engine: tenant-prefixed metrics (reference ``:45-56``)."""

    def __init__(self, name: str | None = None):
        super().__init__(name)
        self.tenant_engine = None

    @property
    def tenant_prefix(self) -> str:
        t = getattr(self.tenant_engine, "tenant", None)
        return f"{t.token}." if t is not None else ""

    def create_meter(self, name: str):
        return self._registry().meter(self.tenant_prefix + name)

    def create_timer(self, name: str):
        return self._registry().timer(self.tenant_prefix + name)

    def create_counter(self, name: str):
        return self._registry().counter(self.tenant_prefix + name)

    def _registry(self):
        from .metrics import MetricRegistry
        ms = self.microservice
        reg = getattr(ms, "metrics", None)
        if reg is None:
            reg = getattr(self, "_local_registry", None)
            if reg is None:
                reg = self._local_registry = MetricRegistry()
        return reg


# ------------------------------------------------------------------------------ steps
class LifecycleStep:
    def __init__(self, name: str):
        self.name = name

    @property
    def operation_count(self) -> int:
        return 1

    def execute(self, monitor: LifecycleProgressMonitor):
        raise NotImplementedError


class SimpleLifecycleStep(LifecycleStep):
    def __init__(self, name: str, fn: Callable[[LifecycleProgressMonitor], None]):
        super().__init__(name)
        self.fn = fn

    def execute(self, monitor):
        self.fn(monitor)


class InitializeComponentLifecycleStep(LifecycleStep):
    def __init__(self, owner: LifecycleComponent, component: LifecycleComponent, name: str | None = None,
                 require: bool = False):
        super().__init__(name or f"Initialize {component.component_name}")
        self.owner, self.component, self.require = owner, component, require

    def execute(self, monitor):
        if self.owner is not None:
            self.owner.initialize_nested_component(self.component, monitor, self.require)
        else:
            self.component.lifecycle_initialize(monitor)
            if self.require and self.component.status == LifecycleStatus.InitializationError:
                raise ServerStartupException(self.component, "initialize failed", self.component.lifecycle_error)


class StartComponentLifecycleStep(LifecycleStep):
    def __init__(self, owner: LifecycleComponent, component: LifecycleComponent, name: str | None = None,
                 require: bool = False):
        super().__init__(name or f"Start {component.component_name}")
        self.owner, self.component, self.require = owner, component, require

    def execute(self, monitor):
        if self.owner is not None:
            self.owner.start_nested_component(self.component, monitor, self.require)
        else:
            self.component.lifecycle_start(monitor)
            if self.require and self.component.status == LifecycleStatus.LifecycleError:
                raise ServerStartupException(self.component, "start failed", self.component.lifecycle_error)


class StopComponentLifecycleStep(LifecycleStep):
    def __init__(self, owner: LifecycleComponent, component: LifecycleComponent, name: str | None = None):
        super().__init__(name or f"Stop {component.component_name}")
        self.owner, self.component = owner, component

    def execute(self, monitor):
        self.component.lifecycle_stop(monitor)


class TerminateComponentLifecycleStep(LifecycleStep):
    def __init__(self, owner: LifecycleComponent, component: LifecycleComponent, name: str | None = None):
        super().__init__(name or f"Terminate {component.component_name}")
        self.owner, self.component = owner, component

    def execute(self, monitor):
        self.component.lifecycle_terminate(monitor)


class CompositeLifecycleStep(LifecycleStep):
    """Ordered steps under one progress context; aborts on the first failure."""

    def __init__(self, name: str, steps: list[LifecycleStep] | None = None):
        super().__init__(name)
        self.steps: list[LifecycleStep] = list(steps or [])

    def add_step(self, step: LifecycleStep) -> "CompositeLifecycleStep":
        self.steps.append(step)
        return self

    def add_initialize_step(self, owner, component, require=False):
        return self.add_step(InitializeComponentLifecycleStep(owner, component, require=require))

    def add_start_step(self, owner, component, require=False):
        return self.add_step(StartComponentLifecycleStep(owner, component, require=require))

    def add_stop_step(self, owner, component):
        return self.add_step(StopComponentLifecycleStep(owner, component))

    def add_terminate_step(self, owner, component):
        return self.add_step(TerminateComponentLifecycleStep(owner, component))

    @property
    def operation_count(self) -> int:
        return sum(s.operation_count for s in self.steps)

    def execute(self, monitor: LifecycleProgressMonitor):
        monitor.push_context(LifecycleProgressContext(len(self.steps), self.name))
        span = monitor.create_tracer_span(self.name)
        try:
            for s in self.steps:
                monitor.start_progress(s.name)
                s.execute(monitor)
                monitor.finish_progress()
        except BaseException as e:
            LifecycleProgressMonitor.handle_error_in_span(span, e)
            raise
        finally:
            LifecycleProgressMonitor.finish_span(span)
            monitor.pop_context()
