"""In-process Azure Event Hubs stand-in speaking AMQP 1.0 (tests and single-node demos).

Serves what ``edges/eventhub.EventHubAmqpReceiver`` (and the Azure SDK's receivers) use:
SASL PLAIN against one SAS key name / key, connection / session setup, a ``$management`` node that
answers the ``READ com.microsoft:eventhub`` query with the partition ids, and partition links
``<hub>/ConsumerGroups/<group>/Partitions/<id>`` positioned by the
``apache.org:selector-filter:string`` offset selector.  Each event carries the ``x-opt-offset``,
``x-opt-sequence-number``, ``x-opt-enqueued-time`` and ``x-opt-partition-key`` annotations and is
sent settled, within the link credit the receiver grants.  ``send(partition, body, key)`` appends
an event, as a device-side producer would.
"""
from __future__ import annotations

import re
import socket
import struct
import threading
import time

from .amqp10 import (AMQP_HEADER, ATTACH, BEGIN, CLOSE, DETACH, END, FLOW, OPEN, SASL_HEADER, SASL_INIT,
                     SASL_MECHANISMS, SASL_OUTCOME, SELECTOR, TRANSFER, Array, Described, Message, Symbol,
                     Timestamp, UByte, UInt, ULong, UShort, decode, encode, frame, perf)

_SEL = re.compile(r"amqp\.annotation\.x-opt-offset\s*(>=|>)\s*'(-?\d+)'")


class _Partition:
    def __init__(self):
        self.events: list[tuple[int, bytes, str | None, int]] = []   # (offset, body, key, enqueued ms)
        self.next_offset = 0


class _Out:
    """A sending link of the server (toward a client receiver)."""

    def __init__(self, handle, remote, partition, start, mgmt=False):
        self.handle, self.remote, self.partition, self.pos, self.mgmt = handle, remote, partition, start, mgmt
        self.credit = 0
        self.delivery_count = 0


class EventHubServer:
    def __init__(self, hub: str = "sitewhere", partitions: int = 4, sas_key_name: str = "RootManageSharedAccessKey",
                 sas_key: str = "secret", host: str = "127.0.0.1", port: int = 0):
        self.hub, self.sas = hub, (sas_key_name, sas_key)
        self.parts = {str(i): _Partition() for i in range(partitions)}
        self._lock = threading.Condition()
        self._srv = socket.create_server((host, port))
        self.address = self._srv.getsockname()
        self._stop = threading.Event()
        self.connections = 0
        self.auth_failures = 0
        self.credited: set = set()          # partitions a receiver link has granted credit on
        self._t = None

    @property
    def port(self) -> int:
        return self.address[1]

    def start(self) -> "EventHubServer":
        self._t = threading.Thread(target=self._accept, daemon=True, name="eventhub-server")
        self._t.start()
        return self

    def stop(self):
        self._stop.set()
        with self._lock:
            self._lock.notify_all()
        try:
            self._srv.close()
        except OSError:
            pass

    def send(self, partition: str, body: bytes, key: str | None = None) -> int:
        with self._lock:
            p = self.parts[str(partition)]
            off = p.next_offset
            p.events.append((off, bytes(body), key, int(time.time() * 1000)))
            p.next_offset += len(body) + 32          # Event Hubs offsets are byte positions, not counts
            self._lock.notify_all()
            return off

    # ---- connections
    def _accept(self):
        while not self._stop.is_set():
            try:
                s, _ = self._srv.accept()
            except OSError:
                return
            self.connections += 1
            threading.Thread(target=self._serve, args=(s,), daemon=True, name="eventhub-conn").start()

    @staticmethod
    def _read_exact(s, n):
        buf = bytearray()
        while len(buf) < n:
            c = s.recv(n - len(buf))
            if not c:
                raise ConnectionError
            buf += c
        return bytes(buf)

    def _read_frame(self, s):
        size, doff, ftype, ch = struct.unpack(">IBBH", self._read_exact(s, 8))
        body = self._read_exact(s, size - 8)[doff * 4 - 8:]
        if not body:
            return None, b"", ch
        p, i = decode(body)
        return p, body[i:], ch

    def _serve(self, s):
        wlock = threading.Lock()

        def send(p, payload=b"", ftype=0):
            with wlock:
                s.sendall(frame(encode(p) + payload, 0, ftype))
        outs: dict[int, _Out] = {}
        ins: dict[int, str] = {}                   # client sender handles -> address
        mgmt_reply = {}
        stop = threading.Event()
        try:
            if self._read_exact(s, 8) != SASL_HEADER:
                return
            s.sendall(SASL_HEADER)
            send(perf(SASL_MECHANISMS, [Array(0xa3, [Symbol("PLAIN"), Symbol("ANONYMOUS")])]), ftype=1)
            p, _, _ = self._read_frame(s)
            mech, resp = str(p.value[0]), p.value[1] or b""
            ok = mech == "PLAIN" and resp.split(b"\x00")[1:] == [x.encode() for x in self.sas]
            if not ok:  # counted before the outcome goes out, so a refused client sees it
                self.auth_failures += 1
            send(perf(SASL_OUTCOME, [UByte(0 if ok else 1)]), ftype=1)
            if not ok:
                return
            if self._read_exact(s, 8) != AMQP_HEADER:
                return
            s.sendall(AMQP_HEADER)
            pump = threading.Thread(target=self._pump, args=(send, outs, stop), daemon=True)
            pump.start()
            next_handle = [0]
            while True:
                p, payload, _ = self._read_frame(s)
                if p is None:
                    continue
                code, f = int(p.descriptor), list(p.value) + [None] * 14
                if code == OPEN:
                    send(perf(OPEN, [f"eventhub-{self.hub}", None, UInt(65536), UShort(0), UInt(60000)]))
                elif code == BEGIN:
                    send(perf(BEGIN, [UShort(0), UInt(0), UInt(65536), UInt(65536), UInt(255)]))
                elif code == ATTACH:
                    name, h, role = f[0], int(f[1]), bool(f[2])
                    src = f[5].value if isinstance(f[5], Described) else None
                    tgt = f[6].value if isinstance(f[6], Described) else None
                    mine = next_handle[0]
                    next_handle[0] += 1
                    if role:                        # client receives: we send
                        addr = (src or [None])[0]
                        filt = (src + [None] * 8)[7] if src else None
                        out = self._open_out(mine, h, addr, filt)
                        if out is None:
                            send(perf(ATTACH, [name, UInt(mine), False, UByte(1), UByte(0), None, tgt and
                                               Described(ULong(0x29), tgt), None, None, UInt(0)]))
                            send(perf(DETACH, [UInt(mine), True, Described(Symbol("amqp:error"), [
                                Symbol("amqp:not-found"), f"no such entity {addr}"])]))
                            continue
                        if out.mgmt:
                            mgmt_reply[name] = out
                        with self._lock:
                            outs[h] = out
                        send(perf(ATTACH, [name, UInt(mine), False, UByte(1), UByte(0),
                                           Described(ULong(0x28), src), Described(ULong(0x29), tgt), None, None,
                                           UInt(0)]))
                    else:                           # client sends (to $management)
                        ins[h] = (tgt or [None])[0]
                        send(perf(ATTACH, [name, UInt(mine), True, UByte(1), UByte(0), Described(ULong(0x28), src),
                                           Described(ULong(0x29), tgt)]))
                        send(perf(FLOW, [UInt(0), UInt(65536), UInt(0), UInt(65536), UInt(mine), UInt(0),
                                         UInt(100)]))
                elif code == FLOW:
                    if f[4] is not None:
                        with self._lock:
                            out = outs.get(int(f[4]))
                            if out is not None:
                                out.credit = int(f[6] or 0)
                                if out.partition is not None and out.credit > 0:
                                    self.credited.add(out.partition)
                                self._lock.notify_all()
                elif code == TRANSFER:
                    if ins.get(int(f[0])) == "$management":
                        req = Message.decode(payload)
                        reply_to = (req.properties + [None] * 6)[4] if req.properties else None
                        msg_id = req.properties[0] if req.properties else None
                        resp = Message(value={"name": self.hub, "partition_count": len(self.parts),
                                              "partition_ids": Array(0xb1, list(self.parts)),
                                              "type": "com.microsoft:eventhub"},
                                       properties=[None, None, None, None, None, msg_id],
                                       app_properties={"status-code": 200})
                        out = next((o for o in outs.values() if o.mgmt), None)
                        if out is not None and reply_to is not None:
                            self._transfer(send, out, resp)
                elif code == DETACH:
                    with self._lock:
                        outs.pop(int(f[0]), None)
                    send(perf(DETACH, [f[0], True]))
                elif code in (END, CLOSE):
                    send(perf(code, []))
                    if code == CLOSE:
                        return
        except (ConnectionError, OSError, ValueError):
            return
        finally:
            stop.set()
            with self._lock:
                self._lock.notify_all()
            try:
                s.close()
            except OSError:
                pass

    def _open_out(self, mine, remote, addr, filt):
        if addr == "$management":
            return _Out(mine, remote, None, 0, mgmt=True)
        m = re.fullmatch(rf"{re.escape(self.hub)}/ConsumerGroups/[^/]+/Partitions/(\w+)", addr or "")
        if m is None or m.group(1) not in self.parts:
            return None
        start = 0
        sel = (filt or {}).get(SELECTOR) if isinstance(filt, dict) else None
        expr = sel.value if isinstance(sel, Described) else sel
        if isinstance(expr, str):
            mm = _SEL.search(expr)
            if mm:
                op, off = mm.group(1), int(mm.group(2))
                evs = self.parts[m.group(1)].events
                start = next((i for i, e in enumerate(evs) if (e[0] >= off if op == ">=" else e[0] > off)), len(evs))
        return _Out(mine, remote, m.group(1), start)

    def _transfer(self, send, out: _Out, msg: Message):
        tag = struct.pack(">I", out.delivery_count)
        send(perf(TRANSFER, [UInt(out.handle), UInt(out.delivery_count), tag, UInt(0), True]), msg.encode())
        out.delivery_count += 1

    def _pump(self, send, outs, stop):
        """Send every partition link the events it has credit for."""
        while not stop.is_set() and not self._stop.is_set():
            work = []
            with self._lock:
                for out in outs.values():
                    if out.mgmt or out.credit <= 0:
                        continue
                    evs = self.parts[out.partition].events
                    while out.credit > 0 and out.pos < len(evs):
                        work.append((out, evs[out.pos]))
                        out.pos += 1
                        out.credit -= 1
                if not work:
                    self._lock.wait(0.2)
                    continue
            for out, (off, body, key, ts) in work:
                ann = {Symbol("x-opt-offset"): str(off), Symbol("x-opt-sequence-number"): off,
                       Symbol("x-opt-enqueued-time"): Timestamp(ts)}
                if key is not None:
                    ann[Symbol("x-opt-partition-key")] = key
                try:
                    self._transfer(send, out, Message(body=body, annotations=ann))
                except OSError:
                    return

