"""Kafka client (wire protocol in :mod:`.kafka_wire`) and :class:`KafkaEventBus`.

* :class:`KafkaClient` -- metadata-routed produce / fetch / list-offsets to partition leaders,
  consumer-group membership through the group coordinator (JoinGroup / SyncGroup / Heartbeat /
  LeaveGroup; the elected leader computes a range assignment, as the Java client does), offset
  commit / fetch, optional TLS and SASL/PLAIN (Azure Event Hubs' Kafka endpoint: user
  ``$ConnectionString``, password = the connection string).
* :class:`KafkaEventBus` -- the :class:`~sitewhere_amd.bus.log.EventBus` surface over a Kafka cluster,
  so every microservice can run on real Kafka exactly as the reference does
  (``MicroserviceKafkaConsumer.java``, ``MicroserviceKafkaProducer.java``), with the Kafka default
  partitioner (murmur2 of the key) routing records to the same partitions.
"""
from __future__ import annotations

import itertools
import socket
import ssl
import struct
import threading
import time
import uuid

from . import kafka_wire as kw
from .log import _FRAME, Consumer, Producer, Record, kafka_partition


class KafkaConnection:
    def __init__(self, host: str, port: int, client_id: str = "sitewhere-amd", tls: ssl.SSLContext | None = None,
                 sasl_plain: tuple[str, str] | None = None, timeout_s: float = 30.0):
        s = socket.create_connection((host, port), timeout=timeout_s)
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self.sock = tls.wrap_socket(s, server_hostname=host) if tls is not None else s
        self.client_id = client_id
        self._corr = itertools.count(1)
        self._lock = threading.Lock()
        if sasl_plain is not None:
            self._sasl_plain(*sasl_plain)

    def _sasl_plain(self, user: str, password: str):
        r = self.request(kw.SASL_HANDSHAKE, {"mechanism": "PLAIN"})
        if r["error_code"]:
            raise kw.KafkaError(r["error_code"], f"SASL mechanisms offered: {r['mechanisms']}")
        r = self.request(kw.SASL_AUTHENTICATE, {"auth_bytes": b"\0" + user.encode() + b"\0" + password.encode()})
        if r["error_code"]:
            raise kw.KafkaError(r["error_code"], r["error_message"] or "SASL authentication failed")

    def request(self, api: int, body: dict, expect_response: bool = True):
        ver = kw.VERSIONS[api]
        with self._lock:
            corr = next(self._corr)
            self.sock.sendall(kw.request_frame(api, ver, corr, self.client_id, kw.encode(kw.REQUEST[api], body)))
            if not expect_response:
                return None
            msg = kw.recv_frame(self.sock)
        (rc,) = struct.unpack_from(">i", msg, 0)
        if rc != corr:
            raise kw.KafkaError(kw.CORRUPT_MESSAGE, f"correlation id {rc} != {corr}")
        return kw.decode(kw.RESPONSE[api], msg, 4)

    def close(self):
        try:
            self.sock.close()
        except OSError:
            pass


def range_assign(members: dict[str, list[str]], partitions: dict[str, int]) -> dict[str, list[tuple[str, int]]]:
    """Kafka's RangeAssignor: per topic, partitions split in contiguous ranges over sorted members."""
    out = {m: [] for m in members}
    for t in sorted({t for ts in members.values() for t in ts}):
        subs = sorted(m for m, ts in members.items() if t in ts)
        n = partitions.get(t, 0)
        per, extra = divmod(n, len(subs))
        p = 0
        for i, m in enumerate(subs):
            c = per + (1 if i < extra else 0)
            out[m].extend((t, q) for q in range(p, p + c))
            p += c
    return out


class KafkaClient:
    def __init__(self, bootstrap: str, client_id: str = "sitewhere-amd", tls: bool | ssl.SSLContext = False,
                 sasl_plain: tuple[str, str] | None = None):
        self.bootstrap = [(h, int(p)) for h, p in (x.rsplit(":", 1) for x in bootstrap.split(","))]
        self.client_id = client_id
        self.tls = (ssl.create_default_context() if tls is True else tls) or None
        self.sasl_plain = sasl_plain
        self._conns: dict = {}
        self._brokers: dict[int, tuple[str, int]] = {}
        self._leaders: dict[tuple[str, int], int] = {}
        self._nparts: dict[str, int] = {}
        self._coord: dict[str, int] = {}
        self._lock = threading.RLock()

    # ------------------------------------------------------------------ connections / metadata
    def _conn(self, node) -> KafkaConnection:
        with self._lock:
            c = self._conns.get(node)
            if c is None:
                host, port = self._brokers[node] if node in self._brokers else self.bootstrap[0]
                c = self._conns[node] = KafkaConnection(host, port, self.client_id, self.tls, self.sasl_plain)
            return c

    def _any(self) -> KafkaConnection:
        return self._conn(next(iter(self._brokers)) if self._brokers else "bootstrap")

    def metadata(self, topics: list[str] | None = None) -> dict[str, int]:
        r = self._any().request(kw.METADATA, {"topics": topics})
        with self._lock:
            for b in r["brokers"]:
                self._brokers[b["node_id"]] = (b["host"], b["port"])
            out = {}
            for t in r["topics"]:
                if t["error_code"]:
                    continue
                out[t["name"]] = len(t["partitions"])
                self._nparts[t["name"]] = len(t["partitions"])
                for p in t["partitions"]:
                    self._leaders[(t["name"], p["partition_index"])] = p["leader_id"]
        return out

    def partitions(self, topic: str) -> int:
        n = self._nparts.get(topic)
        if n is None:
            self.metadata([topic])
            n = self._nparts.get(topic, 0)
        return n

    def _leader(self, topic: str, p: int) -> KafkaConnection:
        node = self._leaders.get((topic, p))
        if node is None:
            self.metadata([topic])
            node = self._leaders[(topic, p)]
        return self._conn(node)

    # ------------------------------------------------------------------ produce / fetch / offsets
    def produce(self, topic: str, partition: int, records, ts: int | None = None, acks: int = 1) -> int:
        """records: [(key, value)] -> base offset (-1 with acks=0)."""
        now = int(time.time() * 1000) if ts is None else int(ts)
        batch = kw.encode_batch([(k, v, now) for k, v in records])
        body = {"transactional_id": None, "acks": acks, "timeout_ms": 30000,
                "topics": [{"name": topic, "partitions": [{"index": partition, "records": batch}]}]}
        r = self._leader(topic, partition).request(kw.PRODUCE, body, expect_response=acks != 0)
        if r is None:
            return -1
        pr = r["responses"][0]["partitions"][0]
        if pr["error_code"]:
            raise kw.KafkaError(pr["error_code"], f"produce {topic}[{partition}]")
        return pr["base_offset"]

    def fetch_many(self, reads, max_wait_ms: int = 500, max_bytes: int = 4 << 20, partition_max_bytes: int = 1 << 20):
        """reads: [(topic, partition, offset)] -> {(topic, p): (records [(offset, key, value, ts)], high watermark,
        error)}; one Fetch per partition leader."""
        by_node: dict = {}
        for t, p, off in reads:
            if (t, p) not in self._leaders:
                self.metadata([t])
            by_node.setdefault(self._leaders[(t, p)], []).append((t, p, off))
        out = {}
        for node, rs in by_node.items():
            topics: dict = {}
            for t, p, off in rs:
                topics.setdefault(t, []).append({"partition": p, "fetch_offset": off,
                                                 "partition_max_bytes": partition_max_bytes})
            body = {"replica_id": -1, "max_wait_ms": max_wait_ms, "min_bytes": 1, "max_bytes": max_bytes,
                    "isolation_level": 0, "topics": [{"topic": t, "partitions": ps} for t, ps in topics.items()]}
            r = self._thread_conn("fetch", node).request(kw.FETCH, body)
            for tr in r["responses"]:
                for pr in tr["partitions"]:
                    recs = kw.decode_batches(pr["records"]) if pr["records"] else []
                    out[(tr["topic"], pr["partition_index"])] = (recs, pr["high_watermark"], pr["error_code"])
        return out

    def list_offset(self, topic: str, partition: int, timestamp: int) -> int:
        body = {"replica_id": -1, "topics": [{"name": topic, "partitions": [{"partition_index": partition,
                                                                             "timestamp": timestamp}]}]}
        pr = self._leader(topic, partition).request(kw.LIST_OFFSETS, body)["topics"][0]["partitions"][0]
        if pr["error_code"]:
            raise kw.KafkaError(pr["error_code"], f"list offsets {topic}[{partition}]")
        return pr["offset"]

    # ------------------------------------------------------------------ groups
    def _coordinator(self, group: str) -> KafkaConnection:
        node = self._coord.get(group)
        if node is None:
            r = self._any().request(kw.FIND_COORDINATOR, {"key": group})
            if r["error_code"]:
                raise kw.KafkaError(r["error_code"], f"coordinator of {group}")
            node = r["node_id"]
            with self._lock:
                self._brokers.setdefault(node, (r["host"], r["port"]))
                self._coord[group] = node
        return self._group_conn(group, node)

    def _thread_conn(self, kind: str, node: int, group: str = "") -> KafkaConnection:
        """Connections for blocking calls are per calling thread: a long-poll Fetch or a JoinGroup that
        waits for a rebalance must not stall other consumers' requests queued on a shared socket."""
        key = (kind, group, node, threading.get_ident())
        with self._lock:
            c = self._conns.get(key)
            if c is None:
                host, port = self._brokers[node]
                c = self._conns[key] = KafkaConnection(host, port, self.client_id, self.tls, self.sasl_plain)
            return c

    def _group_conn(self, group: str, node: int) -> KafkaConnection:
        return self._thread_conn("group", node, group)

    def join_group(self, group: str, topics: list[str], member_id: str = "", session_ms: int = 10000,
                   rebalance_ms: int = 15000):
        """-> (generation, member_id, [(topic, partition)]).  Runs JoinGroup then SyncGroup; the elected
        leader computes the range assignment for everyone."""
        conn = self._coordinator(group)
        meta = kw.encode(kw.SUBSCRIPTION, {"version": 0, "topics": list(topics), "user_data": None})
        while True:
            r = conn.request(kw.JOIN_GROUP, {"group_id": group, "session_timeout_ms": session_ms,
                                             "rebalance_timeout_ms": rebalance_ms, "member_id": member_id,
                                             "protocol_type": "consumer",
                                             "protocols": [{"name": "range", "metadata": meta}]})
            if r["error_code"] == kw.UNKNOWN_MEMBER_ID and member_id:
                member_id = ""
                continue
            if r["error_code"]:
                raise kw.KafkaError(r["error_code"], f"join {group}")
            member_id, gen = r["member_id"], r["generation_id"]
            assignments = []
            if r["leader"] == member_id:
                subs = {m["member_id"]: kw.decode(kw.SUBSCRIPTION, m["metadata"])["topics"] for m in r["members"]}
                parts = {t: self.partitions(t) for ts in subs.values() for t in ts}
                plan = range_assign(subs, parts)
                for m, tps in plan.items():
                    by_t: dict = {}
                    for t, p in tps:
                        by_t.setdefault(t, []).append(p)
                    assignments.append({"member_id": m, "assignment": kw.encode(kw.ASSIGNMENT, {
                        "version": 0, "partitions": [{"topic": t, "partitions": ps} for t, ps in by_t.items()],
                        "user_data": None})})
            s = conn.request(kw.SYNC_GROUP, {"group_id": group, "generation_id": gen, "member_id": member_id,
                                             "assignments": assignments})
            if s["error_code"] in (kw.REBALANCE_IN_PROGRESS, kw.ILLEGAL_GENERATION):
                continue
            if s["error_code"]:
                raise kw.KafkaError(s["error_code"], f"sync {group}")
            mine = []
            if s["assignment"]:
                a = kw.decode(kw.ASSIGNMENT, s["assignment"])
                mine = [(x["topic"], p) for x in a["partitions"] for p in x["partitions"]]
            return gen, member_id, sorted(mine)

    def heartbeat(self, group: str, generation: int, member_id: str) -> int:
        return self._coordinator(group).request(kw.HEARTBEAT, {"group_id": group, "generation_id": generation,
                                                               "member_id": member_id})["error_code"]

    def leave_group(self, group: str, member_id: str):
        self._coordinator(group).request(kw.LEAVE_GROUP, {"group_id": group, "member_id": member_id})

    def commit(self, group: str, offsets, generation: int = -1, member_id: str = ""):
        by_t: dict = {}
        for t, p, off in offsets:
            by_t.setdefault(t, []).append({"partition_index": p, "committed_offset": off, "committed_metadata": None})
        r = self._coordinator(group).request(kw.OFFSET_COMMIT, {
            "group_id": group, "generation_id": generation, "member_id": member_id, "retention_time_ms": -1,
            "topics": [{"name": t, "partitions": ps} for t, ps in by_t.items()]})
        for tr in r["topics"]:
            for pr in tr["partitions"]:
                if pr["error_code"]:
                    raise kw.KafkaError(pr["error_code"], f"commit {group} {tr['name']}[{pr['partition_index']}]")

    def committed(self, group: str, topic: str, partition: int) -> int:
        r = self._coordinator(group).request(kw.OFFSET_FETCH, {"group_id": group, "topics": [
            {"name": topic, "partition_indexes": [partition]}]})
        return r["topics"][0]["partitions"][0]["committed_offset"]

    def close(self):
        with self._lock:
            for c in self._conns.values():
                c.close()
            self._conns.clear()


class _Membership:
    __slots__ = ("kafka_id", "generation", "assignment", "topics", "last_hb")

    def __init__(self, kafka_id, generation, assignment, topics):
        self.kafka_id, self.generation, self.assignment, self.topics = kafka_id, generation, assignment, topics
        self.last_hb = time.time()


class KafkaEventBus:
    """The EventBus surface over a Kafka cluster (or :class:`~.kafka_broker.KafkaBrokerServer`)."""

    def __init__(self, bootstrap: str, client_id: str = "sitewhere-amd", tls: bool | ssl.SSLContext = False,
                 sasl_plain: tuple[str, str] | None = None, heartbeat_s: float = 1.0, session_ms: int = 10000):
        self.client = KafkaClient(bootstrap, client_id, tls, sasl_plain)
        self.heartbeat_s, self.session_ms = heartbeat_s, session_ms
        self._members: dict[tuple[str, str], _Membership] = {}
        self._lock = threading.RLock()
        self.directory = None

    # topics
    def topic(self, name: str, partitions: int | None = None) -> int:
        self.client.partitions(name)          # metadata request auto-creates on the broker
        return 0

    def partitions(self, name: str) -> int:
        return self.client.partitions(name)

    def topics(self) -> list[str]:
        return sorted(self.client.metadata(None))

    def end_offset(self, name: str, p: int) -> int:
        return self.client.list_offset(name, p, -1)

    def begin_offset(self, name: str, p: int) -> int:
        return self.client.list_offset(name, p, -2)

    _rr = itertools.count()

    def partition_for(self, name: str, key: bytes | None) -> int:
        n = self.partitions(name)
        return next(self._rr) % n if key is None else kafka_partition(bytes(key), n)

    # produce
    def append(self, name: str, p: int, records, ts: int | None = None) -> int:
        return self.client.produce(name, p, records, ts) if records else -1

    def append_many(self, batches, ts: int | None = None):
        for name, p, recs in batches:
            self.append(name, p, recs, ts)

    # fetch
    def read(self, name: str, p: int, offset: int, max_records: int = 500, max_bytes: int = 1 << 20):
        got = self.client.fetch_many([(name, p, offset)], max_wait_ms=0, partition_max_bytes=max_bytes)
        recs, _, err = got.get((name, p), ([], -1, 0))
        if err and err != kw.OFFSET_OUT_OF_RANGE:
            raise kw.KafkaError(err, f"fetch {name}[{p}]")
        return [Record(name, p, o, k, v if v is not None else b"", ts) for o, k, v, ts in recs
                if o >= offset][:max_records]

    def fetch_raw(self, reads, max_records: int, timeout_s: float, group=None, member=None):
        """Consumer round trip: group heartbeat, then one Fetch per leader (see EventBus.fetch_raw)."""
        gen = 0
        if group:
            before = self._members.get((group, member))
            gen = self.heartbeat(group, member)
            if before is None or gen != before.generation:
                return -2, []
        if not reads:
            time.sleep(min(timeout_s, 0.1))
            return gen, []
        got = self.client.fetch_many(list(reads), max_wait_ms=int(1000 * min(timeout_s, 1.0)))
        out, budget = [], max_records
        for t, p, off in reads:
            recs = [r for r in got.get((t, p), ([], -1, 0))[0] if r[0] >= off][:max(budget, 0)]
            if not recs:
                continue
            budget -= len(recs)
            buf = bytearray()
            for o, k, v, ts in recs:
                k = k or b""
                v = v if v is not None else b""
                buf += _FRAME.pack(o, ts, len(k), len(v)) + k + v
            out.append((t, p, len(recs), bytes(buf)))
        return gen, out

    def wait_topics(self, topics, timeout_s: float) -> bool:
        time.sleep(min(timeout_s, 0.05))
        return False

    # offsets
    def _gen_member(self, group: str):
        for (g, _), m in self._members.items():
            if g == group:
                return m.generation, m.kafka_id
        return -1, ""

    def commit(self, group: str, name: str, p: int, offset: int):
        self.commit_many(group, [(name, p, offset)])

    def commit_many(self, group: str, offsets):
        gen, mid = self._gen_member(group)
        try:
            self.client.commit(group, list(offsets), gen, mid)
        except kw.KafkaError as e:
            if e.code not in (kw.ILLEGAL_GENERATION, kw.UNKNOWN_MEMBER_ID, kw.REBALANCE_IN_PROGRESS):
                raise
            # a rebalance took the partitions away: the next owner re-reads from the last commit

    def committed(self, group: str, name: str, p: int) -> int:
        return self.client.committed(group, name, p)

    def set_retention(self, name: str, retention_bytes: int):
        """Retention is the Kafka cluster's topic configuration."""

    def retain_from(self, name: str, p: int, offset: int) -> int:
        return self.begin_offset(name, p)

    # group membership (our member ids map to Kafka-assigned ones)
    def join(self, group: str, member_id: str, topics: list[str]) -> int:
        with self._lock:
            old = self._members.get((group, member_id))
            gen, kid, asg = self.client.join_group(group, list(topics), old.kafka_id if old else "",
                                                   self.session_ms, max(self.session_ms, 15000))
            self._members[(group, member_id)] = _Membership(kid, gen, asg, list(topics))
            return gen

    def leave(self, group: str, member_id: str):
        with self._lock:
            m = self._members.pop((group, member_id), None)
        if m is not None:
            try:
                self.client.leave_group(group, m.kafka_id)
            except (kw.KafkaError, OSError):
                pass

    def heartbeat(self, group: str, member_id: str) -> int:
        m = self._members.get((group, member_id))
        if m is None:
            return -1
        if time.time() - m.last_hb < self.heartbeat_s:
            return m.generation
        err = self.client.heartbeat(group, m.generation, m.kafka_id)
        m.last_hb = time.time()
        if err in (kw.REBALANCE_IN_PROGRESS, kw.ILLEGAL_GENERATION, kw.UNKNOWN_MEMBER_ID):
            return self.join(group, member_id, m.topics)
        if err:
            raise kw.KafkaError(err, f"heartbeat {group}")
        return m.generation

    def assignment(self, group: str, member_id: str):
        m = self._members.get((group, member_id))
        return (-1, []) if m is None else (m.generation, list(m.assignment))

    def group_members(self, group: str) -> list[str]:
        return sorted(mid for (g, mid) in self._members if g == group)

    # clients
    def producer(self) -> Producer:
        return Producer(self)

    def consumer(self, group: str, topics: list[str], auto_offset_reset: str = "earliest",
                 member_id: str | None = None) -> Consumer:
        return Consumer(self, group, topics, auto_offset_reset, member_id or f"{group}-{uuid.uuid4().hex[:8]}")

    def flush(self):
        pass

    def close(self):
        with self._lock:
            for (g, mid) in list(self._members):
                self.leave(g, mid)
        self.client.close()
