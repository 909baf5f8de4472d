"""Azure Event Hubs receiver over AMQP 1.0 (the reference's ``EventProcessorHost`` path).

Reference: ``service-event-sources/.../azure/EventHubInboundEventReceiver.java:60-174``: an
``EventProcessorHost`` built from namespace, event hub, consumer group, SAS key name / key and a host
name prefix reads every partition of the hub and checkpoints partition offsets to Azure blob
storage; each event body is handed to the event source's decoder.

Here (``edges/amqp10.py`` underneath):

* the partitions are read from the hub's ``$management`` node (``READ`` of
  ``com.microsoft:eventhub``), or taken from ``partitionCount``;
* one receiving link per owned partition on
  ``<hub>/ConsumerGroups/<group>/Partitions/<id>``, positioned with the
  ``apache.org:selector-filter:string`` offset selector after the partition's checkpoint;
* partition ownership: an ephemeral lease per partition in the coordination store, so several
  event-sources replicas (hosts, ``hostNamePrefix``) split the partitions as EventProcessorHost's
  blob leases do; a host takes over a partition whose owner's session ended;
* checkpoints (the last offset handed to the event source, per consumer group and partition) in the
  coordination store instead of a storage account, written every ``checkpointEvery`` events and on
  stop: after a restart a partition resumes after its checkpoint (at-least-once, as the reference).
"""
from __future__ import annotations

import json
import threading
import time
import uuid

from .amqp10 import SELECTOR, AmqpConnection, AmqpError, Described, Message, Symbol
from .receivers import Receiver


class MemoryCheckpoints:
    """Checkpoint + lease store without coordination (tests, stand-alone receivers)."""

    def __init__(self):
        self.offsets: dict[str, str] = {}
        self.leases: dict[str, str] = {}
        self.members: set[str] = set()
        self._lock = threading.Lock()

    def register(self, owner: str):
        self.members.add(owner)

    def unregister(self, owner: str):
        self.members.discard(owner)

    def hosts(self) -> list[str]:
        return sorted(self.members)

    def get(self, partition: str):
        return self.offsets.get(partition)

    def put(self, partition: str, offset: str):
        self.offsets[partition] = offset

    def acquire(self, partition: str, owner: str) -> bool:
        with self._lock:
            if self.leases.get(partition) in (None, owner):
                self.leases[partition] = owner
                return True
            return False

    def release(self, partition: str, owner: str):
        with self._lock:
            if self.leases.get(partition) == owner:
                del self.leases[partition]


class CoordCheckpoints:
    """Checkpoints (persistent nodes) and leases (ephemeral nodes) under ``base`` in the
    coordination store (ZooKeeper / the in-process store)."""

    def __init__(self, coord, base: str):
        self.coord, self.base = coord, base.rstrip("/")
        self.session = coord.open_session()       # leases vanish with it (a crashed host's partitions free up)

    def get(self, partition: str):
        d = self.coord.get_data(f"{self.base}/checkpoints/{partition}")
        return json.loads(d)["offset"] if d else None

    def put(self, partition: str, offset: str):
        self.coord.put(f"{self.base}/checkpoints/{partition}",
                       json.dumps({"offset": offset, "ts": int(time.time() * 1000)}).encode())

    def acquire(self, partition: str, owner: str) -> bool:
        from ..coord.store import NodeExistsError
        path = f"{self.base}/leases/{partition}"
        try:
            self.coord.create(path, owner.encode(), ephemeral=True, session=self.session)
            return True
        except NodeExistsError:
            d = self.coord.get_data(path)
            return d is not None and d.decode() == owner

    def register(self, owner: str):
        from ..coord.store import NodeExistsError
        try:
            self.coord.create(f"{self.base}/hosts/{owner}", b"", ephemeral=True, session=self.session)
        except NodeExistsError:
            pass

    def unregister(self, owner: str):
        try:
            self.coord.delete(f"{self.base}/hosts/{owner}")
        except KeyError:
            pass

    def hosts(self) -> list[str]:
        try:
            return sorted(self.coord.children(f"{self.base}/hosts"))
        except KeyError:
            return []

    def release(self, partition: str, owner: str):
        path = f"{self.base}/leases/{partition}"
        d = self.coord.get_data(path)
        if d is not None and d.decode() == owner:
            self.coord.delete(path)

    def close(self):
        self.coord.close_session(self.session)


def offset_filter(offset: str | None, inclusive: bool = False) -> dict:
    """Source filter positioning a partition link after (or at) ``offset`` ("-1": the start)."""
    op = ">=" if inclusive else ">"
    expr = f"amqp.annotation.x-opt-offset {op} '{offset if offset is not None else '-1'}'"
    return {SELECTOR: Described(SELECTOR, expr)}


class EventHubAmqpReceiver(Receiver):
    def __init__(self, namespace: str | None, event_hub: str, sas_key_name: str, sas_key: str,
                 consumer_group: str = "$Default", host: str | None = None, port: int = 5671, tls: bool = True,
                 host_name_prefix: str = "sitewhere", partition_count: int | None = None, credit: int = 300,
                 checkpoint_every: int = 100, checkpoints=None, rebalance_s: float = 5.0):
        super().__init__(f"eventhub-receiver:{event_hub}")
        self.host = host or f"{namespace}.servicebus.windows.net"
        self.port, self.tls = port, tls
        self.hub, self.group = event_hub, consumer_group
        self.sas = (sas_key_name, sas_key)
        self.owner = f"{host_name_prefix}-{uuid.uuid4().hex[:8]}"
        self.partition_count, self.credit = partition_count, credit
        self.checkpoint_every, self.rebalance_s = checkpoint_every, rebalance_s
        self.checkpoints = checkpoints
        self.conn: AmqpConnection | None = None
        self.links: dict[str, object] = {}
        self.last_offset: dict[str, str] = {}
        self._since: dict[str, int] = {}
        self._stop = threading.Event()
        self._lock = threading.Lock()
        self._t = None
        self.partitions: list[str] = []
        self._owned: set = set()            # partitions this host reads (set before their link attaches)

    # ---- discovery
    def partition_ids(self) -> list[str]:
        if self.partition_count:
            return [str(i) for i in range(int(self.partition_count))]
        reply = f"$management-reply-{uuid.uuid4().hex[:8]}"
        got, ev = {}, threading.Event()

        def on_reply(msg, _f):
            got["m"] = msg
            ev.set()
        rx = self.conn.attach_receiver("$management", credit=1, on_message=on_reply, name=reply)
        tx = self.conn.attach_sender("$management")
        tx.send(Message(value=None, body=b"", properties=[str(uuid.uuid4()), None, None, None, reply],
                        app_properties={"operation": "READ", "name": self.hub, "type": "com.microsoft:eventhub"}))
        if not ev.wait(self.conn.timeout):
            raise AmqpError("$management did not answer the partition query")
        tx.detach()
        rx.detach()
        v = got["m"].value or {}
        ids = v.get("partition_ids") or v.get(Symbol("partition_ids")) or []
        ids = ids.items if hasattr(ids, "items") and not isinstance(ids, dict) else ids
        return [str(x) for x in ids]

    # ---- lifecycle
    def start(self, monitor):
        if self.checkpoints is None:
            self.checkpoints = self._coord_checkpoints() or MemoryCheckpoints()
        self.conn = AmqpConnection(self.host, self.port, ("PLAIN",) + self.sas, tls=self.tls).open()
        self.partitions = self.partition_ids()
        self.checkpoints.register(self.owner)
        self._stop.clear()
        self._claim()
        self._t = threading.Thread(target=self._balance, daemon=True, name=f"eventhub-{self.hub}")
        self._t.start()

    def _coord_checkpoints(self):
        eng = getattr(self, "tenant_engine", None)
        ms = getattr(eng, "ms", None) if eng is not None else None
        inst = getattr(ms, "instance", None)
        if inst is None:
            return None
        base = inst.tenant_conf_path(eng.tenant.token, "event-sources",
                                     f"eventhub/{self.host}/{self.hub}/{self.group}".replace("$", "_"))
        return CoordCheckpoints(inst.coord, base)

    def _claim(self):
        """Own a fair share of the partitions (EventProcessorHost lease balancing): hand back the
        excess when hosts join, take free partitions up to the share."""
        share = -(-len(self.partitions) // max(1, len(self.checkpoints.hosts())))
        while len(self.links) > share:
            p = sorted(self.links)[-1]
            self._owned.discard(p)
            lk = self.links.pop(p)
            with self._lock:
                if p in self.last_offset:
                    self.checkpoints.put(p, self.last_offset[p])
            lk.detach()
            self.checkpoints.release(p, self.owner)
        for p in self.partitions:
            if len(self.links) >= share:
                break
            if p in self.links or not self.checkpoints.acquire(p, self.owner):
                continue
            start = self.checkpoints.get(p)
            addr = f"{self.hub}/ConsumerGroups/{self.group}/Partitions/{p}"
            # owned before the attach: the hub may deliver as soon as the link has credit, before
            # attach_receiver returns on this thread
            self._owned.add(p)
            self.links[p] = self.conn.attach_receiver(addr, offset_filter(start), self.credit,
                                                      on_message=lambda m, f, p=p: self._on_event(p, m))

    def _on_event(self, p: str, msg: Message):
        if p not in self._owned:
            return                          # handed to another host: it resumes from the checkpoint
        ann = msg.annotations or {}
        off = ann.get(Symbol("x-opt-offset"), ann.get("x-opt-offset"))
        md = {"partition": p, "offset": off, "sequenceNumber": ann.get(Symbol("x-opt-sequence-number")),
              "partitionKey": ann.get(Symbol("x-opt-partition-key")),
              "enqueuedTime": ann.get(Symbol("x-opt-enqueued-time")), "eventHub": self.hub}
        self.deliver(msg.body if msg.body is not None else str(msg.value).encode(), md)
        lk = self.links.get(p)
        with self._lock:
            if off is not None:
                self.last_offset[p] = str(off)
            n = self._since[p] = self._since.get(p, 0) + 1
            if n >= self.checkpoint_every:
                self._since[p] = 0
                self.checkpoints.put(p, self.last_offset[p])
        if lk is not None and lk.credit <= self.credit // 2:
            lk.flow(self.credit)                    # keep the sender's window open

    def checkpoint(self):
        with self._lock:
            for p, off in self.last_offset.items():
                self.checkpoints.put(p, off)
                self._since[p] = 0

    def _balance(self):
        while not self._stop.wait(self.rebalance_s):
            try:
                self.checkpoint()
                if self.conn is not None and not self.conn.closed:
                    self._claim()
            except Exception as e:  # noqa: BLE001 -- keep the receiver alive; log and retry
                self.logger.warning("event hub rebalance failed: %s", e)

    def stop(self, monitor):
        self._stop.set()
        if self._t:
            self._t.join(5)
        self.checkpoint()
        for p in list(self.links):
            self.checkpoints.release(p, self.owner)
        self._owned.clear()
        self.links.clear()
        self.checkpoints.unregister(self.owner)
        if self.conn is not None:
            self.conn.close()
        if hasattr(self.checkpoints, "close"):
            self.checkpoints.close()
