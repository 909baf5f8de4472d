"""The MI355X engine on the event bus without host copies.

The reference moves every event through Kafka topics: event sources produce to
``event-source-decoded-events``, inbound processing consumes it, and enriched events are produced to
``inbound-enriched-events`` for the downstream consumer groups.  Here whole micro-batches move
through the native commit log (``bus/log.py``) in place:

* **raw batches in.**  A producer (event sources, or the bench's synthetic fleet) frames a batch of
  device payloads into one pinned host buffer laid out as a commit-log record
  (:class:`RawBatchRecord`) and publishes it with ``EventBus.append_external``: the log references
  the buffer instead of copying it.  The engine's consumer reads the record in place
  (:func:`raw_view`) and the copy engine DMAs the payload bytes and their varint lengths straight
  from the topic to HBM.  A retention hold covers the records whose H2D is still in flight.
* **enriched rows out.**  :class:`OutboundPublisher` hands the runner a pinned buffer
  (``PipelinedRunner(out_target=...)``); the copy engine writes the step's 32-byte rows into it
  behind a 64-byte batch header and the buffer is published to the enriched-batch topic as is.  Retention
  returns released buffers to the publisher's pool, so the topic's retention window bounds the
  pinned memory and a lagging reader is the only thing that can make the pool grow.

Record formats (little endian, 64-byte headers so the payload and row regions stay aligned):

* raw batch value: ``b"SWRB", version, n_msgs, payload_bytes, payload_off, lens_bytes, lens_off``
  then the payload bytes (plus 64 zero bytes the decoder may over-read) and the LEB128 varint length
  of every payload (``pipeline/framing.py``);
* enriched batch value: ``b"SWOB", version, n_rows, rank, world, step, now_ms`` then ``n_rows``
  :data:`~sitewhere_amd.models.columnar.OUT_REC` rows.
"""
from __future__ import annotations

import ctypes
import struct

import numpy as np

from ..bus.log import EventBus
from ..models.columnar import OUT_REC
from .._native import native
from .framing import varint_lengths

RAW_MAGIC = b"SWRB"
OUT_MAGIC = b"SWOB"
VALUE_HDR = 64
_RAW = struct.Struct("<4sIIIIII")
_OUT = struct.Struct("<4sIIIIqq")
_PAD = 64


_PINNED = None


def partition_payloads(payloads: list, n_partitions: int) -> np.ndarray:
    """Kafka key partition of each raw device payload by its device token (native
    ``sw_partition_payloads``: ``toPositive(murmur2(token)) % n``); -1 where no token parses.
    Event sources split raw batches with it so every device's payloads reach one partition, and
    so one engine replica, as the reference keys decoded events by device token."""
    from .fleet import pack_messages
    from .._native import native
    out = np.zeros(len(payloads), np.int32)
    if not payloads:
        return out
    raw, offs = pack_messages([bytes(p) for p in payloads])
    native().sw_partition_payloads(raw.ctypes.data, offs.ctypes.data, len(payloads), int(n_partitions),
                                   out.ctypes.data)
    return out


def pinned_available() -> bool:
    """Pinned (DMA-able) host memory is there when a GPU runtime is (checked once)."""
    global _PINNED
    if _PINNED is None:
        try:
            import torch
            _PINNED = bool(torch.cuda.is_available())
        except Exception:  # noqa: BLE001
            _PINNED = False
    return _PINNED


class RawBatchRecord:
    """A framed raw batch: the value of one raw-payload topic record, in pinned host memory when
    ``pinned`` (torch's caching host allocator, so steady-state batches reuse pinned blocks)."""

    def __init__(self, payload: np.ndarray, lens: np.ndarray, n_msgs: int, pinned: bool = True):
        payload = np.ascontiguousarray(payload, np.uint8)
        lens = np.ascontiguousarray(lens, np.uint8)
        self.n_msgs = int(n_msgs)
        self.payload_bytes = int(payload.size)
        p_off = VALUE_HDR
        l_off = p_off + self.payload_bytes + _PAD
        self.value_len = l_off + int(lens.size)
        if pinned:
            import torch
            self.buf = torch.empty(self.value_len, dtype=torch.uint8, pin_memory=True)
            a = self.buf.numpy()
            self.ptr = self.buf.data_ptr()
        else:
            self.buf = a = np.empty(self.value_len, np.uint8)
            self.ptr = a.ctypes.data
        a[:VALUE_HDR] = np.frombuffer(_RAW.pack(RAW_MAGIC, 1, self.n_msgs, self.payload_bytes, p_off,
                                                int(lens.size), l_off).ljust(VALUE_HDR, b"\0"), np.uint8)
        a[p_off:p_off + self.payload_bytes] = payload
        a[p_off + self.payload_bytes:l_off] = 0
        a[l_off:l_off + lens.size] = lens

    @classmethod
    def from_payloads(cls, payloads: list, pinned: bool | None = None) -> "RawBatchRecord":
        lens = np.fromiter(map(len, payloads), np.int64, len(payloads))
        offs = np.zeros(len(payloads) + 1, np.int64)
        np.cumsum(lens, out=offs[1:])
        return cls(np.frombuffer(b"".join(payloads), np.uint8), varint_lengths(offs), len(payloads),
                   pinned_available() if pinned is None else pinned)

    def value(self) -> bytes:
        """The record value as bytes (a copy: for buses that cannot publish in place)."""
        return ctypes.string_at(self.ptr, self.value_len)

    def publish(self, bus: EventBus, topic: str, partition: int = 0, ts: int | None = None) -> int:
        return bus.append_external(topic, partition, self, self.ptr, self.value_len, ts=ts)


class RawBatch:
    """A raw batch read from a record value (bytes, or a zero-copy view of the topic): payload bytes
    (with 64 bytes of padding), varint lengths or u32 offsets."""
    __slots__ = ("n_msgs", "payload_bytes", "payload", "lens", "_offs")

    def __init__(self, n_msgs, payload_bytes, payload, lens=None, offs=None):
        self.n_msgs, self.payload_bytes, self.payload, self.lens, self._offs = \
            n_msgs, payload_bytes, payload, lens, offs

    _ERR = {-1: "truncated varint length stream", -2: "over-long varint length",
            -3: "length count does not match the payload count", -4: "lengths do not sum to the payload bytes"}

    def offsets(self) -> np.ndarray:
        """u32 offsets [n + 1] of the payloads, validating the framing (one native pass; the numpy
        form, ``framing.offsets_from_varint``, is the reference)."""
        if self._offs is None:
            if self.n_msgs < 0:
                raise ValueError("corrupt raw batch header")
            offs = np.empty(self.n_msgs + 1, np.uint32)
            lens = np.ascontiguousarray(self.lens, np.uint8)
            rc = native().sw_varint_offsets(lens.ctypes.data if len(lens) else None, len(lens), self.n_msgs,
                                            self.payload_bytes, offs.ctypes.data)
            if rc:
                raise ValueError(f"raw batch framing mismatch: {self._ERR.get(rc, rc)} "
                                 f"({self.n_msgs} payloads of {self.payload_bytes} bytes)")
            self._offs = offs
        return self._offs

    def validate(self):
        """Raise ValueError unless the framing is self-consistent (checked before a batch is stepped:
        a record that fails here is a poison record, dead-lettered instead of retried)."""
        if self.n_msgs < 0 or self.payload_bytes < 0 or len(self.payload) < self.payload_bytes:
            raise ValueError("corrupt raw batch header")
        self.offsets()

    def copy(self) -> "RawBatch":
        """Detached copy (the record's memory may be released once the step is done)."""
        return RawBatch(self.n_msgs, self.payload_bytes, np.array(self.payload), None, self.offsets().copy())


class _SegView:
    """Byte slicing across the parts of a :class:`MultiRawBatch` (names are read from the payload
    bytes by offset; a name never spans two payloads, so never two parts)."""
    __slots__ = ("parts", "starts")

    def __init__(self, parts, starts):
        self.parts, self.starts = parts, starts

    def __getitem__(self, sl):
        a, b = sl.start, sl.stop
        k = int(np.searchsorted(self.starts, a, side="right")) - 1
        base = int(self.starts[k])
        return bytes(self.parts[k].payload[a - base:b - base])


class MultiRawBatch:
    """Consecutive raw batches of one partition stepped as one (the raw consumer coalesces records
    that are already waiting, so small micro-batches share one engine step's fixed cost).  The GPU
    engine DMAs each part's payload and varint lengths back to back (``parts``); host engines and
    the slow path see the concatenation (``payload`` is materialised on first use)."""

    def __init__(self, parts: list):
        self.parts = list(parts)
        self.n_msgs = sum(b.n_msgs for b in self.parts)
        self.payload_bytes = sum(b.payload_bytes for b in self.parts)
        self.starts = np.cumsum([0] + [b.payload_bytes for b in self.parts[:-1]]).astype(np.int64)
        self.msg_starts = np.cumsum([0] + [b.n_msgs for b in self.parts[:-1]]).astype(np.int64)
        self.lens = np.concatenate([np.asarray(b.lens, np.uint8) for b in self.parts]) \
            if all(b.lens is not None for b in self.parts) else None
        self._payload = None
        self._offs = None

    @property
    def payload(self) -> np.ndarray:
        if self._payload is None:
            out = np.zeros(self.payload_bytes + _PAD, np.uint8)
            for b, st in zip(self.parts, self.starts):
                out[st:st + b.payload_bytes] = np.asarray(b.payload)[:b.payload_bytes]
            self._payload = out
        return self._payload

    def host_view(self):
        return _SegView(self.parts, self.starts)

    def offsets(self) -> np.ndarray:
        if self._offs is None:
            offs = np.empty(self.n_msgs + 1, np.uint32)
            for b, st, ms in zip(self.parts, self.starts, self.msg_starts):
                offs[ms:ms + b.n_msgs + 1] = b.offsets() + np.uint32(st)
            self._offs = offs
        return self._offs

    def validate(self):
        for b in self.parts:
            b.validate()

    def copy(self) -> "MultiRawBatch":
        return MultiRawBatch([b.copy() for b in self.parts])


def host_view(batch):
    """What name lookups slice: the payload array, or a segmented view of a coalesced batch."""
    hv = getattr(batch, "host_view", None)
    return hv() if hv is not None else np.asarray(batch.payload)


def parse_raw_batch(value) -> RawBatch:
    """A raw-payload record value: the framed ``SWRB`` form, or the legacy ``u32 n, u32 lengths[n],
    bytes`` form (records written by older event sources / remote producers)."""
    mv = memoryview(value).cast("B")
    if len(mv) >= _RAW.size and bytes(mv[:4]) == RAW_MAGIC:
        magic, ver, n, pb, poff, lb, loff = _RAW.unpack_from(mv, 0)
        if ver != 1 or loff + lb > len(mv) or poff + pb + _PAD > loff:
            raise ValueError("corrupt raw batch record")
        a = np.frombuffer(mv, np.uint8)
        return RawBatch(n, pb, a[poff:poff + pb + _PAD], lens=a[loff:loff + lb])
    (n,) = struct.unpack_from("<I", mv, 0)
    lens = np.frombuffer(mv, np.uint32, n, 4)
    offs = np.zeros(n + 1, np.uint32)
    np.cumsum(lens, out=offs[1:])
    start = 4 + 4 * n
    raw = np.zeros(int(offs[-1]) + _PAD, np.uint8)
    raw[:offs[-1]] = np.frombuffer(mv, np.uint8, int(offs[-1]), start)
    return RawBatch(n, int(offs[-1]), raw, offs=offs)


def _host_tensor(addr: int, n: int):
    import torch
    return torch.frombuffer((ctypes.c_uint8 * n).from_address(addr), dtype=torch.uint8)


def raw_view(view):
    """(payload incl. padding, varint lengths, n_msgs, payload bytes) of a raw-batch record read in
    place -- CPU tensors over the topic's own (pinned) memory, ready for a non-blocking H2D."""
    addr, vlen, _ = view
    magic, ver, n, pb, poff, lb, loff = _RAW.unpack(ctypes.string_at(addr, _RAW.size))
    if magic != RAW_MAGIC or ver != 1 or loff + lb > vlen or poff + pb + _PAD > loff:
        raise ValueError("not a framed raw batch record")
    return _host_tensor(addr + poff, pb + _PAD), _host_tensor(addr + loff, lb), n, pb


class _OutBuf:
    __slots__ = ("host", "nbytes", "hb")

    def __init__(self, hb):
        self.hb, self.host, self.nbytes = hb, hb.host, hb.nbytes


class OutboundPublisher:
    """Pinned row buffers for ``PipelinedRunner(out_target=..., on_outbound=...)`` that become
    enriched-batch records of ``topic`` in place."""

    def __init__(self, bus: EventBus, topic: str, lib, row_capacity: int, partition: int = 0, rank: int = 0,
                 world: int = 1, max_buffers: int = 32, retention_bytes: int | None = None):
        from .gpu_engine import HostBuffer
        self._HostBuffer = HostBuffer
        self.bus, self.topic, self.lib, self.partition = bus, topic, lib, partition
        self.rank, self.world = rank, world
        self.nbytes = VALUE_HDR + row_capacity * OUT_REC.itemsize
        self.max_buffers = max_buffers
        self.free: list[_OutBuf] = []
        self.n_alloc = 0
        self.step = 0
        self.published = 0
        self.rows = 0
        self.now_ms = 0
        bus.topic(topic, partition + 1)
        # the topic keeps about two full batches by default; older records release their buffers
        bus.set_retention(topic, 2 * self.nbytes if retention_bytes is None else int(retention_bytes))

    def _acquire(self) -> _OutBuf:
        if not self.free:
            self.bus.reclaim()              # released row buffers come back through on_release
        if self.free:
            return self.free.pop()
        if self.n_alloc >= self.max_buffers:
            raise RuntimeError(f"enriched-batch buffers exhausted ({self.max_buffers}): a hold or a reader keeps "
                               f"{self.topic} from releasing them")
        self.n_alloc += 1
        return _OutBuf(self._HostBuffer(self.lib, self.nbytes))

    def target(self, nbytes: int):
        """Runner hook: (address the rows are copied to, token)."""
        if VALUE_HDR + nbytes > self.nbytes:
            raise ValueError(f"{nbytes} row bytes exceed the outbound buffer ({self.nbytes})")
        ob = self._acquire()
        return ob.host + VALUE_HDR, ob

    def publish(self, ob: _OutBuf, n_rows: int):
        """Runner hook: the rows are in ``ob``; write the value header and publish the record."""
        hdr = _OUT.pack(OUT_MAGIC, 1, int(n_rows), self.rank, self.world, self.step, int(self.now_ms))
        ctypes.memmove(ob.host, hdr, len(hdr))
        total = VALUE_HDR + int(n_rows) * OUT_REC.itemsize
        self.bus.append_external(self.topic, self.partition, ob, ob.host, total, ts=int(self.now_ms) or None,
                                 on_release=self.free.append)
        self.step += 1
        self.published += 1
        self.rows += int(n_rows)


def read_out_batch(value: bytes) -> tuple[dict, np.ndarray]:
    """Decode an enriched-batch record value (a copy read through ``EventBus.read``)."""
    magic, ver, n, rank, world, step, now = _OUT.unpack_from(value, 0)
    if magic != OUT_MAGIC or ver != 1:
        raise ValueError("not an enriched-batch record")
    rows = np.frombuffer(value, OUT_REC, n, VALUE_HDR)
    return {"rank": rank, "world": world, "step": step, "now": now}, rows
