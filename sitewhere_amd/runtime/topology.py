"""Instance topology (who is alive where) and client-side service discovery / load balancing.

Reference:
  * ``state/TopologyStateAggregator.java:113-160, 278-330`` -- every process consumes all state
    updates and keeps identifier -> hostname -> tenant engines.  **Addition**: members whose
    heartbeats stop are evicted after ``eviction_s`` (the reference only evicts on an explicit
    Terminated message, so crashed replicas stay selectable -- SURVEY §5.3).
  * ``sitewhere-grpc-client/.../ApiDemux.java:80-220`` -- one channel per discovered host,
    round-robin with re-verification, exponential backoff 100 ms -> 3 s while waiting;
    ``MultitenantApiDemux.java:46-71`` -- per-channel tenant-engine availability cache (5 s).
"""
from __future__ import annotations

import itertools
import json
import threading
import time
from dataclasses import dataclass, field

from ..core.errors import SiteWhereException, TenantEngineNotAvailableException
from ..core.lifecycle import LifecycleComponent, LifecycleStatus


class NoLiveReplicaException(SiteWhereException):
    """No replica of the target microservice is in the topology (yet)."""


@dataclass
class TenantEngineState:
    tenant: str
    status: str
    updated: float = field(default_factory=time.time)


@dataclass
class MicroserviceState:
    identifier: str
    hostname: str
    status: str
    api_address: str | None = None
    last_seen: float = field(default_factory=time.time)
    tenant_engines: dict = field(default_factory=dict)


class TopologySnapshot:
    def __init__(self):
        self.by_identifier: dict[str, dict[str, MicroserviceState]] = {}

    def hosts(self, identifier: str) -> list[MicroserviceState]:
        return sorted(self.by_identifier.get(identifier, {}).values(), key=lambda s: s.hostname)

    def to_dict(self) -> dict:
        return {ident: {h: {"status": s.status, "apiAddress": s.api_address, "lastSeen": s.last_seen,
                            "tenantEngines": {t: e.status for t, e in s.tenant_engines.items()}}
                        for h, s in hosts.items()} for ident, hosts in self.by_identifier.items()}


class TopologyStateAggregator(LifecycleComponent):
    """Consumes ``microservice-state-updates`` (unique consumer group per process -> sees all)."""

    TERMINAL = (LifecycleStatus.Terminating.value, LifecycleStatus.Terminated.value)

    def __init__(self, bus, topic: str, member: str, eviction_s: float = 60.0):
        super().__init__("topology-aggregator")
        self.bus, self.topic, self.member = bus, topic, member
        self.eviction_s = eviction_s
        self.snapshot = TopologySnapshot()
        self._lock = threading.RLock()
        self._topo_listeners = []
        self._stop = threading.Event()
        self._t = None

    def add_listener(self, cb):
        """cb(kind, state) with kind in {'added', 'updated', 'removed'}."""
        self._topo_listeners.append(cb)

    def _notify(self, kind, st):
        for cb in list(self._topo_listeners):
            try:
                cb(kind, st)
            except Exception:
                self.logger.exception("topology listener failed")

    def apply(self, msg: dict):
        ident, host = msg["identifier"], msg["hostname"]
        with self._lock:
            hosts = self.snapshot.by_identifier.setdefault(ident, {})
            cur = hosts.get(host)
            if msg.get("type") == "tenant":
                if cur is None:
                    cur = hosts[host] = MicroserviceState(ident, host, LifecycleStatus.Started.value)
                    self._notify("added", cur)
                cur.tenant_engines[msg["tenant"]] = TenantEngineState(msg["tenant"], msg["status"])
                cur.last_seen = time.time()
                self._notify("updated", cur)
                return
            if msg["status"] in self.TERMINAL:
                if cur is not None:
                    del hosts[host]
                    self._notify("removed", cur)
                return
            if cur is None:
                cur = hosts[host] = MicroserviceState(ident, host, msg["status"], msg.get("apiAddress"))
                self._notify("added", cur)
            else:
                cur.status = msg["status"]
                cur.api_address = msg.get("apiAddress") or cur.api_address
                cur.last_seen = time.time()
                self._notify("updated", cur)

    def evict_stale(self, now: float | None = None) -> list[MicroserviceState]:
        now = now or time.time()
        gone = []
        with self._lock:
            for ident, hosts in self.snapshot.by_identifier.items():
                for h in [h for h, s in hosts.items() if now - s.last_seen > self.eviction_s]:
                    gone.append(hosts.pop(h))
        for s in gone:
            self._notify("removed", s)
        return gone

    def start(self, monitor):
        self._consumer = self.bus.consumer(f"topology-{self.member}", [self.topic], auto_offset_reset="earliest")
        self._stop.clear()
        self._t = threading.Thread(target=self._run, daemon=True, name=f"topology-{self.member}")
        self._t.start()

    def _run(self):
        while not self._stop.is_set():
            batch = self._consumer.poll(200)
            for recs in batch.values():
                for r in recs:
                    try:
                        self.apply(json.loads(r.value))
                    except Exception:
                        self.logger.exception("bad state update")
            self.evict_stale()

    def stop(self, monitor):
        self._stop.set()
        if self._t:
            self._t.join(timeout=2)
        if getattr(self, "_consumer", None):
            self._consumer.close()

    def wait_for(self, identifier: str, timeout_s: float = 10.0, tenant: str | None = None) -> bool:
        end = time.time() + timeout_s
        while time.time() < end:
            with self._lock:
                for s in self.snapshot.hosts(identifier):
                    if s.status in (LifecycleStatus.Started.value, LifecycleStatus.StartedWithErrors.value):
                        if tenant is None or (tenant in s.tenant_engines and
                                              s.tenant_engines[tenant].status == LifecycleStatus.Started.value):
                            return True
            time.sleep(0.02)
        return False


class ApiDemux:
    """Round-robin over the channels of every live replica of one microservice identifier."""

    def __init__(self, identifier: str, topology: TopologyStateAggregator, channel_factory, local_channel=None,
                 availability_ttl_s: float = 5.0):
        self.identifier = identifier
        self.topology = topology
        self.factory = channel_factory          # api_address -> ApiChannel
        self.local = local_channel              # in-process fallback (co-located services)
        self.ttl = availability_ttl_s
        self._channels: dict[str, object] = {}
        self._rr = itertools.count()
        self._avail: dict[tuple[str, str], float] = {}
        self._lock = threading.RLock()
        topology.add_listener(self._on_topology)
        for s in topology.snapshot.hosts(identifier):
            self._on_topology("added", s)

    def _on_topology(self, kind, st: MicroserviceState):
        if st.identifier != self.identifier:
            return
        with self._lock:
            if kind == "removed":
                ch = self._channels.pop(st.hostname, None)
                if ch is not None:
                    ch.close()
            elif st.api_address and st.hostname not in self._channels:
                self._channels[st.hostname] = self.factory(st.api_address)

    def channels(self) -> list:
        with self._lock:
            return [self._channels[h] for h in sorted(self._channels)]

    def get_channel(self, tenant: str | None = None):
        chans = self.channels()
        if not chans:
            if self.local is not None:
                return self.local
            raise NoLiveReplicaException(f"no live replica of {self.identifier}")
        n = len(chans)
        start = next(self._rr)
        for i in range(n):
            ch = chans[(start + i) % n]
            if tenant is None or self._tenant_available(ch, tenant):
                return ch
        raise TenantEngineNotAvailableException(f"{self.identifier}: no replica has tenant {tenant} available")

    def _tenant_available(self, ch, tenant: str) -> bool:
        key = (id(ch), tenant)
        t = self._avail.get(key)
        if t and time.time() - t < self.ttl:
            return True
        try:
            ok = bool(ch.call("MultitenantManagement", "CheckTenantEngineAvailable", tenant, tenant=tenant))
        except Exception:
            ok = False
        if ok:
            self._avail[key] = time.time()
        return ok

    def wait_for_available(self, timeout_s: float = 30.0, tenant: str | None = None):
        """Exponential backoff 100 ms -> 3 s (reference ApiDemux.waitForMicroserviceAvailable)."""
        delay, end = 0.1, time.time() + timeout_s
        while True:
            try:
                return self.get_channel(tenant)
            except SiteWhereException:
                if time.time() >= end:
                    raise
                time.sleep(delay)
                delay = min(3.0, delay * 2)

    def proxy(self, service: str, tenant: str | None = None):
        demux = self

        class _P:
            def __getattr__(self, name):
                def call(*args, **kwargs):
                    ch = demux.get_channel(tenant)
                    return ch.proxy(service, tenant).__getattr__(name)(*args, **kwargs)
                return call
        return _P()
