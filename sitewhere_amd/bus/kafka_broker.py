"""Kafka-protocol front end for the native commit log: any Kafka client can produce to and consume
from a SiteWhere-AMD bus.

Reference: the reference services talk to Apache Kafka through kafka-clients
(``MicroserviceKafkaProducer.java:41-107``, ``MicroserviceKafkaConsumer.java:53-133``); with this
server a reference service, a device gateway that writes to Kafka, or Kafka tooling
(console consumer, Connect, MirrorMaker) can be pointed at the rebuilt bus unchanged.

One broker node (id 0) owns every partition.  Topics, offsets and committed group offsets are the
:class:`~sitewhere_amd.bus.log.EventBus` ones, so Kafka clients and in-process services share the
same streams and consumer groups.  The group coordinator implements the Kafka group protocol
(JoinGroup / SyncGroup / Heartbeat / LeaveGroup): members are assigned partitions by their elected
leader, exactly as with a real broker.  Optional SASL/PLAIN authentication (``users``).
Each API is served at one version (``kafka_wire.VERSIONS``), which clients from 0.11 through 3.x
negotiate through ApiVersions; clients that dropped those versions (4.x removed JoinGroup v0-v1)
are refused at negotiation rather than misunderstood.

    srv = KafkaBrokerServer(bus, port=9092).start()
"""
from __future__ import annotations

import logging
import socket
import socketserver
import threading
import time
import uuid

from . import kafka_wire as kw

log = logging.getLogger(__name__)


class _Member:
    __slots__ = ("member_id", "client_id", "protocols", "session_ms", "rebalance_ms", "last_hb")

    def __init__(self, member_id, client_id, protocols, session_ms, rebalance_ms):
        self.member_id, self.client_id = member_id, client_id
        self.protocols, self.session_ms, self.rebalance_ms = protocols, session_ms, rebalance_ms
        self.last_hb = time.time()


class _Group:
    """Kafka group state machine: Empty -> PreparingRebalance -> AwaitingSync -> Stable."""

    def __init__(self, gid: str, cond: threading.Condition):
        self.gid = gid
        self.cond = cond
        self.members: dict[str, _Member] = {}
        self.state = "Empty"
        self.generation = 0
        self.leader: str | None = None
        self.protocol_type: str | None = None
        self.protocol: str | None = None
        self.assignments: dict[str, bytes] = {}
        self.joined: set = set()
        self.round = 0
        self.deadline = 0.0

    # all under self.cond
    def start_rebalance(self, rebalance_ms: int):
        if self.state != "PreparingRebalance":
            self.state = "PreparingRebalance"
            self.joined = set()
            self.deadline = time.time() + max(rebalance_ms, 1000) / 1000.0
        self.cond.notify_all()

    def try_complete(self, force: bool = False):
        if self.state != "PreparingRebalance":
            return
        if not (force or set(self.members) <= self.joined):
            return
        for m in list(self.members):
            if m not in self.joined:
                del self.members[m]                      # did not rejoin within the rebalance timeout
        self.generation += 1
        self.round += 1
        self.assignments = {}
        if not self.members:
            self.state, self.leader, self.protocol = "Empty", None, None
        else:
            if self.leader not in self.members:
                self.leader = next(iter(self.members))
            common = None
            for name, _ in self.members[self.leader].protocols:
                if all(any(n == name for n, _ in m.protocols) for m in self.members.values()):
                    common = name
                    break
            self.protocol = common
            self.state = "AwaitingSync"
        self.cond.notify_all()


class _Handler(socketserver.BaseRequestHandler):
    def handle(self):
        srv: KafkaBrokerServer = self.server.broker        # type: ignore[attr-defined]
        sock: socket.socket = self.request
        sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        authed = not srv.users
        sasl_ok_handshake = False
        try:
            while not srv._stop.is_set():
                msg = kw.recv_frame(sock)
                api, ver, corr, client_id, pos = kw.parse_request_header(msg)
                if api == kw.API_VERSIONS:
                    body = srv.api_versions(ver)
                elif api == kw.SASL_HANDSHAKE:
                    req = kw.decode(kw.REQUEST[api], msg, pos)
                    ok = req["mechanism"] == "PLAIN"
                    sasl_ok_handshake = ok
                    body = kw.encode(kw.RESPONSE[api], {"error_code": kw.NONE if ok else kw.UNSUPPORTED_SASL_MECHANISM,
                                                        "mechanisms": ["PLAIN"]})
                elif api == kw.SASL_AUTHENTICATE:
                    req = kw.decode(kw.REQUEST[api], msg, pos)
                    code, why = kw.ILLEGAL_SASL_STATE, "handshake first"
                    if sasl_ok_handshake:
                        parts = req["auth_bytes"].split(b"\0")
                        user, pw = (parts[1].decode(), parts[2].decode()) if len(parts) == 3 else ("", "")
                        ok = bool(srv.users) and srv.users.get(user) == pw
                        code, why = (kw.NONE, None) if ok else (kw.SASL_AUTHENTICATION_FAILED, "bad credentials")
                        authed = authed or ok
                    body = kw.encode(kw.RESPONSE[api], {"error_code": code, "error_message": why, "auth_bytes": b""})
                elif not authed:
                    log.warning("unauthenticated kafka request %d from %s", api, self.client_address)
                    return
                elif kw.VERSIONS.get(api) != ver:
                    log.warning("unsupported kafka api %d v%d from %s", api, ver, client_id)
                    return                                  # Kafka closes the connection too
                else:
                    req = kw.decode(kw.REQUEST[api], msg, pos)
                    res = srv.dispatch(api, req, client_id or "")
                    if res is None:                         # produce with acks=0: no response
                        continue
                    body = kw.encode(kw.RESPONSE[api], res)
                sock.sendall(kw.response_frame(corr, body))
        except (ConnectionError, OSError):
            pass
        except kw.KafkaError as e:
            log.warning("kafka connection %s dropped: %s", self.client_address, e)


class _Server(socketserver.ThreadingTCPServer):
    daemon_threads = True
    allow_reuse_address = True


class KafkaBrokerServer:
    def __init__(self, bus, host: str = "127.0.0.1", port: int = 9092, advertised_host: str | None = None,
                 users: dict[str, str] | None = None):
        self.bus = bus
        self.users = dict(users or {})
        self._srv = _Server((host, port), _Handler)
        self._srv.broker = self
        self.host = advertised_host or host
        self.port = self._srv.server_address[1]
        self._lock = threading.RLock()
        self._cond = threading.Condition(self._lock)
        self._groups: dict[str, _Group] = {}
        self._stop = threading.Event()

    @property
    def address(self) -> str:
        return f"{self.host}:{self.port}"

    def start(self):
        threading.Thread(target=self._srv.serve_forever, daemon=True, name="kafka-broker").start()
        threading.Thread(target=self._reaper, daemon=True, name="kafka-group-reaper").start()
        return self

    def stop(self):
        self._stop.set()
        self._srv.shutdown()
        self._srv.server_close()
        with self._cond:
            self._cond.notify_all()

    # ------------------------------------------------------------------ dispatch
    def api_versions(self, ver: int) -> bytes:
        keys = [{"api_key": k, "min_version": v, "max_version": v} for k, v in sorted(kw.VERSIONS.items())]
        # a newer client probing with a flexible ApiVersions gets the v0 body + UNSUPPORTED_VERSION
        return kw.encode(kw.RESPONSE[kw.API_VERSIONS], {"error_code": kw.NONE if ver == 0 else kw.UNSUPPORTED_VERSION,
                                                        "api_keys": keys})

    def dispatch(self, api: int, req: dict, client_id: str):
        return {
            kw.METADATA: self._metadata, kw.PRODUCE: self._produce, kw.FETCH: self._fetch,
            kw.LIST_OFFSETS: self._list_offsets, kw.FIND_COORDINATOR: self._find_coordinator,
            kw.JOIN_GROUP: lambda r: self._join(r, client_id), kw.SYNC_GROUP: self._sync,
            kw.HEARTBEAT: self._heartbeat, kw.LEAVE_GROUP: self._leave, kw.OFFSET_COMMIT: self._offset_commit,
            kw.OFFSET_FETCH: self._offset_fetch,
        }[api](req)

    def _metadata(self, req):
        names = self.bus.topics() if req["topics"] is None else req["topics"]
        topics = []
        for n in names:
            self.bus.topic(n)                             # auto-create, as the reference relied on
            parts = [{"error_code": kw.NONE, "partition_index": p, "leader_id": 0, "replica_nodes": [0],
                      "isr_nodes": [0]} for p in range(self.bus.partitions(n))]
            topics.append({"error_code": kw.NONE, "name": n, "is_internal": False, "partitions": parts})
        return {"brokers": [{"node_id": 0, "host": self.host, "port": self.port, "rack": None}],
                "controller_id": 0, "topics": topics}

    def _produce(self, req):
        out = []
        for t in req["topics"]:
            name = t["name"]
            self.bus.topic(name)
            parts = []
            for pd in t["partitions"]:
                p = pd["index"]
                code, base = kw.NONE, -1
                if not 0 <= p < self.bus.partitions(name):
                    code = kw.UNKNOWN_TOPIC_OR_PARTITION
                else:
                    try:
                        recs = kw.decode_batches(pd["records"])
                        if recs:
                            base = self.bus.append(name, p, [(k, v if v is not None else b"") for _, k, v, _ in recs],
                                                   ts=recs[0][3])
                    except kw.KafkaError as e:
                        code = e.code
                parts.append({"index": p, "error_code": code, "base_offset": base, "log_append_time_ms": -1})
            out.append({"name": name, "partitions": parts})
        if req["acks"] == 0:
            return None
        return {"responses": out, "throttle_time_ms": 0}

    def _read_partition(self, name, p, off, max_bytes):
        if not 0 <= p < self.bus.partitions(name):
            return kw.UNKNOWN_TOPIC_OR_PARTITION, -1, None
        end = self.bus.end_offset(name, p)
        if off < self.bus.begin_offset(name, p) or off > end:
            return kw.OFFSET_OUT_OF_RANGE, end, None
        if off == end:
            return kw.NONE, end, None
        recs = self.bus.read(name, p, off, 10_000, max(1024, max_bytes))
        if not recs:
            return kw.NONE, end, None
        batch = kw.encode_batch([(r.key, r.value, r.timestamp) for r in recs], base_offset=recs[0].offset)
        return kw.NONE, end, batch

    def _fetch(self, req):
        topics = {t["topic"] for t in req["topics"]}
        for n in topics:
            self.bus.topic(n)
        ev = threading.Event()
        local = hasattr(self.bus, "subscribe_event")
        if local:
            self.bus.subscribe_event(topics, ev)          # before the first read: no lost wake-up
        deadline = time.time() + max(0, req["max_wait_ms"]) / 1000.0
        try:
            while True:
                ev.clear()
                out, got = [], 0
                budget = req["max_bytes"] if req["max_bytes"] > 0 else 1 << 30
                for t in req["topics"]:
                    parts = []
                    for pd in t["partitions"]:
                        code, hw, batch = kw.NONE, -1, None
                        if budget > 0:
                            code, hw, batch = self._read_partition(t["topic"], pd["partition"], pd["fetch_offset"],
                                                                   min(pd["partition_max_bytes"], budget))
                        else:
                            hw = self.bus.end_offset(t["topic"], pd["partition"])
                        if batch:
                            got += len(batch)
                            budget -= len(batch)
                        parts.append({"partition_index": pd["partition"], "error_code": code, "high_watermark": hw,
                                      "last_stable_offset": hw, "aborted_transactions": None, "records": batch})
                    out.append({"topic": t["topic"], "partitions": parts})
                left = deadline - time.time()
                if got >= max(1, req["min_bytes"]) or left <= 0 or self._stop.is_set():
                    return {"throttle_time_ms": 0, "responses": out}
                if local:
                    ev.wait(min(left, 0.5))
                else:
                    self.bus.wait_topics(list(topics), min(left, 0.5))
        finally:
            if local:
                self.bus.unsubscribe_event(topics, ev)

    def _offset_for_time(self, name, p, ts):
        lo, hi = self.bus.begin_offset(name, p), self.bus.end_offset(name, p)
        while lo < hi:                                    # first offset with timestamp >= ts
            mid = (lo + hi) // 2
            r = self.bus.read(name, p, mid, 1)
            if r and r[0].timestamp < ts:
                lo = mid + 1
            else:
                hi = mid
        return lo

    def _list_offsets(self, req):
        out = []
        for t in req["topics"]:
            name = t["name"]
            self.bus.topic(name)
            parts = []
            for pd in t["partitions"]:
                p, ts = pd["partition_index"], pd["timestamp"]
                if not 0 <= p < self.bus.partitions(name):
                    parts.append({"partition_index": p, "error_code": kw.UNKNOWN_TOPIC_OR_PARTITION, "timestamp": -1,
                                  "offset": -1})
                    continue
                if ts == -1:
                    off = self.bus.end_offset(name, p)
                elif ts == -2:
                    off = self.bus.begin_offset(name, p)
                else:
                    off = self._offset_for_time(name, p, ts)
                parts.append({"partition_index": p, "error_code": kw.NONE, "timestamp": -1, "offset": off})
            out.append({"name": name, "partitions": parts})
        return {"topics": out}

    def _find_coordinator(self, req):
        return {"error_code": kw.NONE, "node_id": 0, "host": self.host, "port": self.port}

    # ------------------------------------------------------------------ group coordinator
    def _group(self, gid) -> _Group:
        g = self._groups.get(gid)
        if g is None:
            g = self._groups[gid] = _Group(gid, self._cond)
        return g

    def _join(self, req, client_id):
        with self._cond:
            g = self._group(req["group_id"])
            mid = req["member_id"]
            if g.protocol_type and g.members and req["protocol_type"] != g.protocol_type:
                return self._join_error(kw.INCONSISTENT_GROUP_PROTOCOL, mid)
            if mid and mid not in g.members:
                return self._join_error(kw.UNKNOWN_MEMBER_ID, mid)
            if not mid:
                mid = f"{client_id or 'consumer'}-{uuid.uuid4()}"
            protocols = [(p["name"], p["metadata"]) for p in req["protocols"]]
            m = g.members.get(mid)
            if m is None:
                g.members[mid] = _Member(mid, client_id, protocols, req["session_timeout_ms"],
                                         req["rebalance_timeout_ms"])
            else:
                m.protocols, m.last_hb = protocols, time.time()
            g.protocol_type = req["protocol_type"]
            g.start_rebalance(req["rebalance_timeout_ms"])
            g.joined.add(mid)
            my_round = g.round
            g.try_complete()
            while g.round == my_round and not self._stop.is_set():
                left = g.deadline - time.time()
                if left <= 0:
                    g.try_complete(force=True)
                    break
                self._cond.wait(min(left, 0.5))
            if mid not in g.members:
                return self._join_error(kw.UNKNOWN_MEMBER_ID, mid)
            members = []
            if mid == g.leader:
                for m in g.members.values():
                    meta = next((md for n, md in m.protocols if n == g.protocol), b"")
                    members.append({"member_id": m.member_id, "metadata": meta})
            return {"error_code": kw.NONE, "generation_id": g.generation, "protocol_name": g.protocol or "",
                    "leader": g.leader or "", "member_id": mid, "members": members}

    @staticmethod
    def _join_error(code, mid):
        return {"error_code": code, "generation_id": -1, "protocol_name": "", "leader": "", "member_id": mid or "",
                "members": []}

    def _sync(self, req):
        with self._cond:
            g = self._group(req["group_id"])
            mid, gen = req["member_id"], req["generation_id"]
            if mid not in g.members:
                return {"error_code": kw.UNKNOWN_MEMBER_ID, "assignment": b""}
            if g.state == "PreparingRebalance":
                return {"error_code": kw.REBALANCE_IN_PROGRESS, "assignment": b""}
            if gen != g.generation:
                return {"error_code": kw.ILLEGAL_GENERATION, "assignment": b""}
            g.members[mid].last_hb = time.time()
            if mid == g.leader and g.state == "AwaitingSync":
                g.assignments = {a["member_id"]: a["assignment"] for a in req["assignments"]}
                g.state = "Stable"
                self._cond.notify_all()
            deadline = time.time() + g.members[mid].session_ms / 1000.0
            while g.state == "AwaitingSync" and g.generation == gen and time.time() < deadline:
                self._cond.wait(0.5)
            if g.generation != gen or g.state != "Stable":
                return {"error_code": kw.REBALANCE_IN_PROGRESS, "assignment": b""}
            return {"error_code": kw.NONE, "assignment": g.assignments.get(mid, b"")}

    def _heartbeat(self, req):
        with self._cond:
            g = self._group(req["group_id"])
            m = g.members.get(req["member_id"])
            if m is None:
                return {"error_code": kw.UNKNOWN_MEMBER_ID}
            m.last_hb = time.time()
            if g.state == "PreparingRebalance":
                return {"error_code": kw.REBALANCE_IN_PROGRESS}
            if req["generation_id"] != g.generation:
                return {"error_code": kw.ILLEGAL_GENERATION}
            return {"error_code": kw.NONE}

    def _leave(self, req):
        with self._cond:
            g = self._group(req["group_id"])
            if g.members.pop(req["member_id"], None) is None:
                return {"error_code": kw.UNKNOWN_MEMBER_ID}
            if g.members:
                g.start_rebalance(max(m.rebalance_ms for m in g.members.values()))
            else:
                g.state, g.leader = "Empty", None
                self._cond.notify_all()
            return {"error_code": kw.NONE}

    def _reaper(self):
        while not self._stop.wait(0.5):
            with self._cond:
                now = time.time()
                for g in self._groups.values():
                    # session expiry; a member blocked in JoinGroup of the current round is alive
                    dead = [m for m in g.members.values() if now - m.last_hb > m.session_ms / 1000.0 and
                            not (g.state == "PreparingRebalance" and m.member_id in g.joined)]
                    for m in dead:
                        del g.members[m.member_id]
                    if dead:
                        if g.members:
                            g.start_rebalance(max(m.rebalance_ms for m in g.members.values()))
                        else:
                            g.state, g.leader = "Empty", None
                    if g.state == "PreparingRebalance":
                        g.try_complete(force=now >= g.deadline)

    def _offset_commit(self, req):
        gid = req["group_id"]
        with self._cond:
            g = self._groups.get(gid)
            gen_ok = (g is None or not g.members or req["generation_id"] < 0 or
                      (req["generation_id"] == g.generation and req["member_id"] in g.members))
        out = []
        for t in req["topics"]:
            parts = []
            for pd in t["partitions"]:
                code = kw.NONE if gen_ok else kw.ILLEGAL_GENERATION
                if gen_ok:
                    self.bus.commit(gid, t["name"], pd["partition_index"], pd["committed_offset"])
                parts.append({"partition_index": pd["partition_index"], "error_code": code})
            out.append({"name": t["name"], "partitions": parts})
        return {"topics": out}

    def _offset_fetch(self, req):
        out = []
        for t in req["topics"] or []:
            parts = [{"partition_index": p, "committed_offset": self.bus.committed(req["group_id"], t["name"], p),
                      "metadata": "", "error_code": kw.NONE} for p in t["partition_indexes"]]
            out.append({"name": t["name"], "partitions": parts})
        return {"topics": out}
