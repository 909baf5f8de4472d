"""Durable columnar event segments: the persistent event store of MI355X (and native CPU) tenants.

Each engine step's persisted events become one *block* (format: ``csrc/include/swseg.h``): ~8 B per
event, frame-of-reference + decimal coded columns, page checksums.  On the MI355X the block is
encoded by ``k_seg_encode`` right after the step and only the compressed block crosses PCIe; host
engines encode the same bytes with :func:`encode_block`.  :class:`SegmentStore` appends blocks to
segment files through the native group-commit writer (``csrc/native/swseg.cpp``: O_DIRECT when the
buffer allows it, one ``fdatasync`` per drained group, torn-tail recovery on open).  A block's token
is durable once its sync returned: input offsets are committed only then (at-least-once across a
crash; replayed blocks are skipped by sequence).

:class:`DurableEventStore` is the ``DeviceEventStore`` over a segment store: it keeps the
dictionaries the rows refer to (assignment index -> ids, name id -> name, rule alert messages) in a
small fsync'd JSON-lines log beside the segments, keeps the events added through the API (REST adds,
command invocations / responses, rule alerts) in a checksummed JSON-lines log synced before the add
returns, answers the event-management queries by decoding
the blocks whose date range overlaps, and survives restarts (everything is reloaded from disk).

Reference: ``DeviceEventBuffer.java:99-135`` (buffered bulk writes, flushed every 250 ms / 200
documents, lost on a crash: ``SURVEY §5.4``) and ``MongoDeviceEventManagement`` (queries by index
and date range).  Here nothing is acknowledged before it is on disk.
"""
from __future__ import annotations

import contextlib
import ctypes
import functools
import json
import os
import threading
import time
import zlib
from collections import OrderedDict

import numpy as np

from .._native import native
from ..models.columnar import (EV_ALERT, EV_COMMAND_INVOCATION, EV_COMMAND_RESPONSE, EV_LOCATION, EV_MEASUREMENT,
                               EV_STATE_CHANGE, NO_NAME, OUT_REC)
from ..models.domain import (AlertLevel, AlertSource, DateRangeSearchCriteria, DeviceAlert, DeviceEventIndex,
                             DeviceEventType, DeviceLocation, DeviceMeasurement, DeviceStateChange, SearchResults,
                             event_from_dict)
from .events import DeviceEventStore, MemoryEventStore

# SEG_FLAGS bits (csrc/include/swseg.h)
SEGF_HAS_US, SEGF_US, SEGF_HAS_ELEV, SEGF_HAS_ALT, SEGF_HAS_META, SEGF_GEN = 0x1, 0x2, 0x4, 0x8, 0x10, 0x20
SEGF_SYS, SEGF_JSON = 0x40, 0x80          # API-added rows: System alert with a message; JSON fields
SEG_ALIGN = 4096
PAGE_ROWS = 1024
PAGE_HDR = 400              # sizeof(SwSegPageHdr), csrc/include/swseg.h
FLAG_COMMIT = 1             # the block is followed by a commit record of input offsets (swseg.h)
FLAG_INDEX = 2              # the block carries its index trailer (swindex.h)
MAX_SRC = 252
HDR = np.dtype([("magic", "<u4"), ("version", "<u2"), ("flags", "<u2"), ("n_rows", "<u4"), ("n_pages", "<u4"),
                ("bytes", "<u8"), ("first_seq", "<i8"), ("recv_ms", "<i8"), ("boot", "<i8"), ("rank", "<i4"),
                ("world", "<i4"), ("checksum", "<u8")])
assert HDR.itemsize == 64
INDEX_ENT = np.dtype([("first_seq", "<i8"), ("recv_ms", "<i8"), ("offset", "<i8"), ("bytes", "<i8"),
                      ("file", "<i4"), ("n_rows", "<i4"), ("rank", "<i4"), ("world", "<i4"),
                      ("min_date", "<i8"), ("max_date", "<i8"), ("boot", "<i8")])
assert INDEX_ENT.itemsize == 72


def _p(a: np.ndarray) -> int:
    return a.ctypes.data


# Block index trailer (csrc/include/swindex.h)
IX_DIMS = 3                         # customer, area, asset
IX_HEADS = 16
IX_CTX_MAX = 8192
IX_NOT_INDEXED = 0xFFFFFFFF
IX_ALT_EBITS = 26
IX_MAGIC = 0x58495753
IX_HDR = np.dtype([("magic", "<u4"), ("version", "<u2"), ("n_dims", "<u2"), ("n_rows", "<u4"), ("n_pages", "<u4"),
                   ("bytes", "<u8"), ("checksum", "<u8"), ("alt_bits", "<u4"), ("alt_pbits", "<u4"), ("n_alt", "<u4"),
                   ("off_pages", "<u4"), ("off_alt_dir", "<u4"), ("off_alt", "<u4"), ("off_keys", "<u4", 3),
                   ("n_keys", "<u4", 3), ("off_heads", "<u4", 3), ("n_heads", "<u4", 3), ("off_hdates", "<u4", 3),
                   ("flags", "<u4"), ("pad", "<u4", 2)])
assert IX_HDR.itemsize == 128
IX_F_CLUSTERED = 1          # SIX_F_CLUSTERED (csrc/include/swindex.h)
IX_PAGE = np.dtype([("asg_min", "<i4"), ("asg_max", "<i4"), ("date_min", "<i8"), ("date_max", "<i8"), ("off", "<u4"),
                    ("bytes", "<u4")])
IX_KEY = np.dtype([("key", "<u4"), ("count", "<u4"), ("date_min", "<i8"), ("date_max", "<i8"), ("head_off", "<u4"),
                   ("n_heads", "<u4")])


def parse_trailer(t) -> dict:
    """Index trailer bytes -> header fields and numpy views of its sections: ``pages`` (IX_PAGE),
    ``alt_dir`` (u32), ``alt_words`` (u64), per dimension ``keys[d]`` (IX_KEY, None: not indexed),
    ``head_rows[d]`` / ``head_dates[d]``."""
    t = np.frombuffer(t, np.uint8) if not isinstance(t, np.ndarray) else t
    h = t[:128].view(IX_HDR)[0]
    d = {k: (h[k].copy() if h[k].shape else int(h[k])) for k in IX_HDR.names}
    d["pages"] = t[d["off_pages"]:d["off_pages"] + 32 * d["n_pages"]].view(IX_PAGE)
    d["alt_dir"] = t[d["off_alt_dir"]:d["off_alt_dir"] + 4 * ((1 << d["alt_bits"]) + 1)].view(np.uint32)
    nw = (d["n_alt"] * IX_ALT_EBITS + 63) // 64
    d["alt_words"] = t[d["off_alt"]:d["off_alt"] + 8 * nw].view(np.uint64)
    d["keys"], d["head_rows"], d["head_dates"] = [], [], []
    for q in range(IX_DIMS):
        nk, nh = int(d["n_keys"][q]), int(d["n_heads"][q])
        if nk == IX_NOT_INDEXED:
            d["keys"].append(None)
            d["head_rows"].append(np.zeros(0, np.uint32))
            d["head_dates"].append(np.zeros(0, np.int64))
            continue
        ok, oh, od = int(d["off_keys"][q]), int(d["off_heads"][q]), int(d["off_hdates"][q])
        d["keys"].append(t[ok:ok + 32 * nk].view(IX_KEY))
        d["head_rows"].append(t[oh:oh + 4 * nh].view(np.uint32))
        d["head_dates"].append(t[od:od + 8 * nh].view(np.int64))
    return d


def alt_entries(tr: dict) -> np.ndarray:
    """The packed alternate-id entries of a parsed trailer, unpacked (u64: fingerprint << pbits | page)."""
    n = tr["n_alt"]
    w = np.concatenate([tr["alt_words"], np.zeros(1, np.uint64)])
    bp = np.arange(n, dtype=np.uint64) * np.uint64(IX_ALT_EBITS)
    wi, sh = (bp >> np.uint64(6)).astype(np.int64), bp & np.uint64(63)
    lo = w[wi] >> sh
    hi = np.where(sh > 0, w[wi + 1] << ((np.uint64(64) - sh) & np.uint64(63)), np.uint64(0))
    return (lo | hi) & np.uint64((1 << IX_ALT_EBITS) - 1)


def max_block_bytes(n_rows: int, string_bytes: int = 0) -> int:
    """Upper bound of an encoded block (every column at 64 bits plus exceptions, every string of the
    rows in the heap: ``string_bytes``), padded."""
    pages = (n_rows + PAGE_ROWS - 1) // PAGE_ROWS
    worst = (64 + 8 * (pages + 2) + pages * (PAGE_HDR + 8 + 16 * 16) + n_rows * (15 * 8 + 4 * 10)
             + 8 * 4 * 15 * pages + int(string_bytes))
    return -(-worst // SEG_ALIGN) * SEG_ALIGN


def max_string_bytes(n_rows: int, raw_bytes: int) -> int:
    """Heap bound of a step's block: every row's strings come from its own payload, so the heap holds
    at most the batch's bytes once per row of a payload -- bounded by 3 x 64 KiB per row and, for
    the usual one row per payload, by the batch itself."""
    return min(3 * 0xFFFF * int(n_rows), 2 * int(raw_bytes) + 64 * int(n_rows)) + 8 * PAGE_ROWS


def encode_block(rows: np.ndarray, recs: np.ndarray | None = None, spans: np.ndarray | None = None,
                 raw: np.ndarray | None = None, index: bool = False, ctx: np.ndarray | None = None) -> np.ndarray:
    """CPU encoder (bit-identical to the MI355X ``k_seg_encode``): OUT_REC rows, each with its
    persisted EVENT_REC record and STR_REF string refs (row-aligned; None: rows without record
    data -- no strings, elevation or flags) into the raw batch ``raw`` -> block bytes (header sealed
    separately by :func:`seal`).  ``index``: append the block's index trailer (``swindex.h``, the
    same bytes the MI355X builds); ``ctx`` = int32 [assignments, 4] (device, customer, area, asset)
    by assignment index, None: the context dimensions stay unindexed."""
    from ..models.columnar import EVENT_REC, STR_REF
    rows = np.ascontiguousarray(rows, OUT_REC)
    n = len(rows)
    if recs is not None:
        recs = np.ascontiguousarray(recs, EVENT_REC)
        assert len(recs) >= n
    if spans is not None:
        spans = np.ascontiguousarray(spans, STR_REF)
        assert len(spans) >= n
    raw_a = None if raw is None else np.ascontiguousarray(raw, np.uint8)
    cap = max_block_bytes(n, 0 if raw_a is None else max_string_bytes(n, len(raw_a)))
    if index:
        cap += int(native().swseg_ix_max_bytes(n))
    out = np.zeros(cap, np.uint8)
    r = native().swseg_encode(_p(rows) if n else None, _p(recs) if recs is not None and n else None,
                              _p(spans) if spans is not None and n else None,
                              _p(raw_a) if raw_a is not None and len(raw_a) else None,
                              0 if raw_a is None else len(raw_a), n, _p(out), cap)
    if r < 0:
        raise RuntimeError(f"block needs {-r} bytes")
    if index:
        r = _index_into(out, cap, ctx)
    return out[:r]


def _index_into(buf: np.ndarray, cap: int, ctx: np.ndarray | None) -> int:
    if ctx is not None:
        ctx = np.ascontiguousarray(ctx, np.int32).reshape(-1, 4)
    r = int(native().swseg_index_append(_p(buf), int(cap), _p(ctx) if ctx is not None and len(ctx) else None,
                                        0 if ctx is None else len(ctx)))
    if r < 0:
        raise RuntimeError(f"block index trailer failed ({r})")
    return r


def index_block(block: np.ndarray, ctx: np.ndarray | None = None) -> np.ndarray:
    """A copy of ``block`` (sealed or not) with its index trailer (rebuilt if it had one)."""
    b = np.ascontiguousarray(block, np.uint8)
    n = int(b[:64].view(HDR)[0]["n_rows"])
    cap = len(b) + int(native().swseg_ix_max_bytes(n))
    out = np.zeros(cap, np.uint8)
    out[:len(b)] = b
    return out[:_index_into(out, cap, ctx)]


def trailer_offset(block) -> int:
    """Offset of a block's index trailer, 0 when it has none."""
    b = np.frombuffer(block, np.uint8) if not isinstance(block, np.ndarray) else block
    return int(native().swseg_ix_offset(_p(np.ascontiguousarray(b[:64 + 4 * (int(b[:64].view(HDR)[0]["n_pages"]) + 2)]))))


def seal(block: np.ndarray, first_seq: int, recv_ms: int, boot: int, rank: int, world: int):
    """Fill the header: the block's first store sequence, receive time and engine incarnation."""
    native().swseg_seal(_p(block), int(first_seq), int(recv_ms), int(boot), int(rank), int(world))


def source_key(topic: str, partition: int) -> int:
    """64-bit key of an input (topic, partition) in commit records (stable across processes)."""
    import hashlib
    return int.from_bytes(hashlib.blake2b(f"{topic}/{int(partition)}".encode(), digest_size=8).digest(), "little")


def set_commit_flag(block: np.ndarray):
    """Mark a sealed block as carrying a commit record (see :meth:`SegmentStore.append`)."""
    native().swseg_set_flags(_p(block), FLAG_COMMIT)


def verify(block) -> int:
    b = np.frombuffer(block, np.uint8) if not isinstance(block, np.ndarray) else block
    return int(native().swseg_verify(_p(b), len(b)))


def header(block) -> dict:
    b = np.frombuffer(block, np.uint8, 64) if not isinstance(block, np.ndarray) else block[:64]
    h = b.view(HDR)[0]
    return {k: int(h[k]) for k in HDR.names}


def decode_block(block, pages: tuple[int, int] | None = None, strings: bool = True, check: bool = True) -> dict:
    """Block -> per-row columns (etype, level, date, asg, name, v0, v1, v2, flags) + header fields,
    and with ``strings`` the rows' alternate ids, alert messages and metadata spans (see
    :func:`row_strings`).  ``pages`` = (first, end) decodes only those pages (rows from the first
    row of ``first``; ``cols["row0"]`` is that row's index in the block)."""
    b = np.ascontiguousarray(np.frombuffer(block, np.uint8) if not isinstance(block, np.ndarray) else block)
    if check:
        rc = verify(b)
        if rc:
            raise ValueError(f"corrupt event block (code {rc})")
    h = header(b)
    lib = native()
    p0, p1 = (0, h["n_pages"]) if pages is None else (max(0, int(pages[0])), min(h["n_pages"], int(pages[1])))
    n = max(0, min(h["n_rows"], p1 * PAGE_ROWS) - p0 * PAGE_ROWS) if p1 > p0 else 0
    cols = {"etype": np.empty(n, np.uint8), "level": np.empty(n, np.uint8), "date": np.empty(n, np.int64),
            "asg": np.empty(n, np.int32), "name": np.empty(n, np.uint16), "v0": np.empty(n, np.float64),
            "v1": np.empty(n, np.float64), "v2": np.empty(n, np.float64), "flags": np.empty(n, np.uint8)}
    heap = offs = None
    if n:
        if strings:
            cap = int(lib.swseg_string_bytes(_p(b), p0, p1))
            heap = np.empty(max(cap, 8), np.uint8)
            offs = np.zeros(3 * n + 1, np.int64)
        got = lib.swseg_decode(_p(b), p0, p1, *[_p(cols[k]) for k in ("etype", "level", "date", "asg", "name", "v0",
                                                                        "v1", "v2", "flags")],
                               _p(heap) if heap is not None else None, 0 if heap is None else len(heap),
                               _p(offs) if offs is not None else None)
        if got != n:
            raise ValueError(f"event block decode failed ({got} of {n} rows)")
    cols["header"] = h
    cols["row0"] = p0 * PAGE_ROWS
    cols["str_heap"], cols["str_off"] = heap, offs
    return cols


def _str(cols: dict, i: int, part: int) -> bytes:
    o = cols["str_off"]
    if o is None:
        return b""
    return cols["str_heap"][o[3 * i + part]:o[3 * i + part + 1]].tobytes()


_META_FIELD = {EV_MEASUREMENT: 4, EV_LOCATION: 6, EV_ALERT: 5}


def parse_metadata(span: bytes, field: int) -> dict:
    """Metadata entries of a body's wire span (``Model.Metadata {name = 1; value = 2}`` as field
    ``field``) -> dict; other fields interleaved in the span are skipped."""
    from ..models.wire import iter_fields
    md = {}
    for f, wt, v in iter_fields(span):
        if f == field and wt == 2:
            name = value = None
            for f2, wt2, v2 in iter_fields(v):
                if f2 == 1 and wt2 == 2:
                    name = v2.decode("utf-8", "replace")
                elif f2 == 2 and wt2 == 2:
                    value = v2.decode("utf-8", "replace")
            if name is not None:
                md[name] = value if value is not None else ""
    return md


def row_strings(cols: dict, i: int) -> tuple[str | None, str, dict]:
    """(alternate id or None, alert message, metadata dict) of decoded row ``i``."""
    f = int(cols["flags"][i])
    alt = _str(cols, i, 0).decode("utf-8", "replace") if f & SEGF_HAS_ALT else None
    msg = _str(cols, i, 1).decode("utf-8", "replace")
    md = parse_metadata(_str(cols, i, 2), _META_FIELD.get(int(cols["etype"][i]), 0)) \
        if f & SEGF_HAS_META and not f & SEGF_JSON else {}
    return alt, msg, md


def rows_of(cols: dict) -> np.ndarray:
    """Decoded columns -> OUT_REC rows (the enriched-row form consumers use)."""
    out = np.zeros(len(cols["date"]), OUT_REC)
    out["event_date"], out["v0"], out["v1"] = cols["date"], cols["v0"], cols["v1"]
    out["assignment"], out["name_id"], out["etype"], out["level"] = cols["asg"], cols["name"], cols["etype"], cols["level"]
    return out


def page_summary(block) -> np.ndarray:
    """Per-page (first row, rows, assignment min, max, date min, max) of a block: the page index."""
    b = np.ascontiguousarray(np.frombuffer(block, np.uint8) if not isinstance(block, np.ndarray) else block)
    n = header(b)["n_pages"]
    out = np.zeros((n, 6), np.int64)
    if n:
        native().swseg_page_summary(_p(b), _p(out))
    return out


# ---------------------------------------------------------------------- durable batch wire format
# What an engine tenant sends event management (and publishes on the enriched-batch topic):
# b"SWD1", u32 header length, msgpack {"boot", "asg", "names", "rules"} (the dictionary deltas the
# rows need), zero padding up to a 64-byte multiple, then the sealed block.  When the block sits at a
# 4 KiB boundary of a pinned buffer the header is framed in front of it (:func:`frame_durable_batch`)
# and the block goes to the disk with O_DIRECT straight from that buffer.
DURABLE_MAGIC = b"SWD1"


def _durable_head(boot, asg: dict, names: dict, rules: dict | None, src=None, ctx=None) -> bytes:
    import msgpack
    import struct
    d = {"boot": boot_id(boot), "asg": {int(k): list(v) for k, v in (asg or {}).items()},
         "names": {int(k): v for k, v in (names or {}).items()}, "rules": rules or {}}
    if src:
        d["src"] = [[str(t), int(p), int(o)] for t, p, o in src]
    if ctx:
        d["ctx"] = {int(k): {str(t): int(i) for t, i in m.items()} for k, m in ctx.items()}
    hdr = msgpack.packb(d, use_bin_type=True)
    head = DURABLE_MAGIC + struct.pack("<I", len(hdr)) + hdr
    return head + bytes(-len(head) % 64)


def encode_durable_batch(block: np.ndarray, boot, asg: dict | None = None, names: dict | None = None,
                         rules: dict | None = None, src=None, ctx: dict | None = None) -> bytes:
    """``src``: ``[(topic, partition, next offset)]`` of the input the block completes (the block
    should then carry ``FLAG_COMMIT``, see :func:`set_commit_flag`); ``ctx``: context-id deltas
    (:meth:`DurableEventStore.add_dictionary`)."""
    return _durable_head(boot, asg, names, rules, src, ctx) + memoryview(np.ascontiguousarray(block, np.uint8)).cast("B")


def frame_durable_batch(frame: tuple, nbytes: int, boot, asg: dict | None = None, names: dict | None = None,
                        rules: dict | None = None, src=None, ctx: dict | None = None) -> np.ndarray | None:
    """Zero-copy :func:`encode_durable_batch` for a block at ``offset`` of ``buffer`` (``frame``)
    with free bytes in front of it; None when the header does not fit."""
    buf, off = frame
    head = _durable_head(boot, asg, names, rules, src, ctx)
    start = off - len(head)
    if start < 0:
        return None
    buf[start:off] = np.frombuffer(head, np.uint8)
    view = buf[start:off + int(nbytes)]
    view.flags.writeable = False
    return view


def is_durable_batch(payload) -> bool:
    return bytes(memoryview(payload)[:4]) == DURABLE_MAGIC


def decode_durable_batch(payload) -> tuple[dict, np.ndarray]:
    """(header dict, block bytes view) of a durable batch (bytes or a zero-copy buffer)."""
    import msgpack
    import struct
    buf = np.frombuffer(payload, np.uint8) if not isinstance(payload, np.ndarray) else payload
    if bytes(buf[:4]) != DURABLE_MAGIC:
        raise ValueError("not a durable event batch")
    (n,) = struct.unpack_from("<I", bytes(buf[4:8]))
    d = msgpack.unpackb(bytes(buf[8:8 + n]), raw=False, strict_map_key=False)
    start = -(-(8 + n) // 64) * 64
    return d, buf[start:]


class SegmentStore:
    """Native durable segment store of one engine shard (see module docstring)."""

    def __init__(self, directory: str, rank: int = 0, rotate_bytes: int = 1 << 30, retention_bytes: int = 0,
                 direct: bool = True):
        os.makedirs(directory, exist_ok=True)
        self.lib = native()
        self.dir = directory
        self.rank = rank
        self.h = self.lib.swss_open(directory.encode(), int(rank), int(rotate_bytes), int(retention_bytes),
                                    1 if direct else 0)
        self._owners: OrderedDict[int, object] = OrderedDict()     # token -> buffer owner (kept until durable)
        self._lock = threading.Lock()
        self._token = int(self.lib.swss_durable(self.h))
        self.closed = False

    def append(self, ptr: int, nbytes: int, owner=None, src=None) -> int:
        """Queue a sealed block at ``ptr`` (``nbytes``, readable up to the next 4 KiB multiple with
        zeroed padding when ``ptr`` is 4 KiB aligned).  ``owner`` is kept alive until the block is
        durable.  ``src``: ``[(topic, partition, next offset)]`` the block completes -- written as a
        commit record with the block (it must carry ``FLAG_COMMIT``), so after a crash the block is
        on disk exactly when these offsets are (:meth:`sources`).  Returns the block's token."""
        if src is not None:
            if len(src) > MAX_SRC:
                raise ValueError("too many input offsets for one commit record")
            keys = np.array([source_key(t, p) for t, p, _ in src], np.uint64)
            offs = np.array([int(o) for _, _, o in src], np.int64)
        with self._lock:
            self._token += 1
            tok = self._token
            self._owners[tok] = owner
            if src is not None:
                rc = self.lib.swss_append_commit(self.h, ptr, int(nbytes), tok, _p(keys) if len(keys) else None,
                                                 _p(offs) if len(offs) else None, len(keys))
            else:
                rc = self.lib.swss_append(self.h, ptr, int(nbytes), tok)
        if rc:
            raise OSError(rc, f"segment store append failed: {os.strerror(rc) if rc > 0 else rc}")
        return tok

    def append_block(self, block: np.ndarray) -> int:
        return self.append(_p(block), len(block), block)

    def sources(self) -> dict:
        """Durable input offsets: source key -> next offset (max over commit records)."""
        cap = 64
        while True:
            keys, offs = np.zeros(cap, np.uint64), np.zeros(cap, np.int64)
            n = int(self.lib.swss_sources(self.h, _p(keys), _p(offs), cap))
            if n <= cap:
                return {int(k): int(o) for k, o in zip(keys[:n], offs[:n])}
            cap = n + 64

    def source_offset(self, topic: str, partition: int) -> int | None:
        return self.sources().get(source_key(topic, partition))

    def durable(self) -> int:
        """Highest token whose block (and every earlier one) is on disk."""
        d = int(self.lib.swss_durable(self.h))
        with self._lock:
            while self._owners and next(iter(self._owners)) <= d:
                self._owners.popitem(last=False)
        err = int(self.lib.swss_error(self.h))
        if err:
            raise OSError(err, f"segment store write failed: {os.strerror(err) if err > 0 else err}")
        return d

    def wait(self, token: int, timeout_s: float = 60.0) -> bool:
        rc = int(self.lib.swss_wait(self.h, int(token), int(timeout_s * 1000)))
        if rc > 0:
            raise OSError(rc, f"segment store write failed: {os.strerror(rc)}")
        self.durable()
        return rc == 0

    def flush(self, timeout_s: float = 60.0) -> bool:
        return self.wait(self._token, timeout_s)

    @property
    def last_token(self) -> int:
        return self._token

    def stats(self) -> dict:
        a = np.zeros(16, np.int64)
        self.lib.swss_stats(self.h, _p(a))
        return dict(zip(("bytes_written", "blocks_written", "syncs", "deleted_files", "deleted_bytes", "retained_bytes",
                         "files", "direct_io", "write_ns", "sync_ns", "copier_wait_ns", "copier_ns", "retained_rows",
                         "deleted_rows", "retention_rows", "retention_bytes"),
                        (int(x) for x in a)))

    def set_retention(self, bytes_: int = 0, rows: int = 0, rotate_bytes: int = 0):
        """Set the retention limits (0: unchanged; rows -1: none) and the size at which new files start
        (0: unchanged); applied after the next group commit."""
        self.lib.swss_set_retention(self.h, int(bytes_), int(rows), int(rotate_bytes))

    def index(self) -> np.ndarray:
        cap = 1024
        while True:
            out = np.zeros(cap, INDEX_ENT)
            n = int(self.lib.swss_index(self.h, _p(out), cap))
            if n <= cap:
                return out[:n]
            cap = n + 1024

    def index_tr(self):
        """(index entries, trailer copy addresses, trailer lengths, block copy addresses): see
        swss_index_tr.  Hold a :meth:`lease` while using the addresses."""
        cap = 1024
        while True:
            out = np.zeros(cap, INDEX_ENT)
            ta, tl, ba = np.zeros(cap, np.uint64), np.zeros(cap, np.int64), np.zeros(cap, np.uint64)
            n = int(self.lib.swss_index_tr(self.h, _p(out), _p(ta), _p(tl), _p(ba), cap))
            if n <= cap:
                return out[:n], ta[:n], tl[:n], ba[:n]
            cap = n + 1024

    def mem_caps(self, trailer_bytes: int = -1, block_bytes: int = -1) -> tuple[int, int]:
        """Set the bytes of index-trailer copies and of recent-block copies the store holds in
        memory (-1: leave); returns the bytes held (trailers, blocks)."""
        held = np.zeros(1, np.int64)
        t = int(self.lib.swss_mem_caps(self.h, int(trailer_bytes), int(block_bytes), _p(held)))
        return t, int(held[0])

    @contextlib.contextmanager
    def lease(self):
        """A read lease: in-memory copies seen through :meth:`index_tr` stay valid until it ends."""
        tok = int(self.lib.swss_lease_begin(self.h))
        try:
            yield tok
        finally:
            self.lib.swss_lease_end(self.h, tok)

    def file_path(self, file_id: int) -> str | None:
        buf = ctypes.create_string_buffer(4096)
        n = self.lib.swss_file(self.h, int(file_id), buf, 4096)
        return None if n < 0 else buf.value.decode()

    def read_block(self, ent) -> np.ndarray:
        path = self.file_path(int(ent["file"]))
        if path is None:
            raise KeyError("segment file deleted by retention")
        with open(path, "rb", buffering=0) as f:
            f.seek(int(ent["offset"]))
            return np.frombuffer(f.read(int(ent["bytes"])), np.uint8)

    def close(self):
        if not self.closed:
            self.closed = True
            self.lib.swss_close(self.h)
            self._owners.clear()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


class _BlockBuf:
    __slots__ = ("hb", "host", "nbytes", "refs", "token")

    def __init__(self, hb):
        self.hb, self.host, self.nbytes = hb, hb.host, hb.nbytes
        self.refs = 0
        self.token = -1


class DurableBlockSink:
    """Pinned, page-aligned host buffers for the MI355X runner's encoded blocks
    (``PipelinedRunner(block_sink=...)``).  Each step's block is DMA'd by the copy engine into one,
    sealed, queued to the durable store (O_DIRECT straight from the buffer) and, with a bus, published
    in place to the enriched-batch topic.  A buffer goes back to the pool once the store has made its
    block durable and the topic's retention has released it.  ``publish`` returns the store token;
    ``committable(tag)`` lists the caller tags (e.g. raw-topic offsets) whose blocks are durable."""

    def __init__(self, store: "DurableEventStore", lib, boot: int, rank: int = 0, world: int = 1, bus=None,
                 topic: str | None = None, partition: int = 0, max_buffers: int = 64):
        from ..pipeline.gpu_engine import HostBuffer
        self._HostBuffer = HostBuffer
        self.store, self.lib, self.boot, self.rank, self.world = store, lib, int(boot), rank, world
        self.bus, self.topic, self.partition = bus, topic, partition
        self.max_buffers = max_buffers
        self.free: list[_BlockBuf] = []
        self.pending: list[_BlockBuf] = []            # queued to the store, not yet durable
        self.tags: list[tuple[int, object]] = []      # (store token, caller tag), in order
        self.n_alloc = 0
        self.blocks = self.bytes = self.rows = 0
        self.index_bytes = 0                          # of which index trailers
        self.disk_wait_s = 0.0                        # time target() waited for the disk (backpressure)
        self._size = 0
        self._lock = threading.Lock()
        if bus is not None and topic is not None:
            bus.topic(topic, partition + 1)

    def _release(self, b: _BlockBuf):
        with self._lock:
            b.refs -= 1
            if b.refs == 0:
                self.free.append(b)

    def _reap(self):
        d = self.store.durable()
        keep = []
        for b in self.pending:
            if b.token <= d:
                self._release(b)
            else:
                keep.append(b)
        self.pending = keep
        if self.bus is not None:
            self.bus.reclaim()

    def target(self, nbytes: int, timeout_s: float = 60.0):
        """(host address, buffer) for a block of ``nbytes`` (the copy engine writes it there).  When
        every buffer is in use the caller waits for the disk (backpressure), never for more memory
        than ``max_buffers`` buffers."""
        import time as _time
        need = -(-int(nbytes) // SEG_ALIGN) * SEG_ALIGN
        deadline = _time.monotonic() + timeout_s
        while True:
            self._reap()
            with self._lock:
                for i, b in enumerate(self.free):
                    if b.nbytes >= need:
                        b = self.free.pop(i)
                        b.refs = 1
                        return b.host, b
                small = self.free.pop(0) if self.free else None
            # buffers only the topic still references are bounded by its retention (bytes), not by
            # the disk: those never count against max_buffers (a reader window of small blocks
            # would otherwise starve the pool, as retention only runs on the next append)
            topic_only = self.n_alloc - len(self.free) - len(self.pending) - 1
            if small is not None or self.n_alloc - max(0, topic_only) < self.max_buffers:
                if small is not None:           # too small for this block: replace it
                    self.n_alloc -= 1
                    del small
                # sized with headroom: steps of one engine produce blocks of about the same size
                self._size = max(self._size, need + need // 2)
                self.n_alloc += 1
                b = _BlockBuf(self._HostBuffer(self.lib, self._size))
                b.refs = 1
                return b.host, b
            if _time.monotonic() > deadline:
                raise RuntimeError(f"durable block buffers exhausted ({self.n_alloc} allocated, {len(self.pending)} "
                                   f"waiting for the disk, durable token {self.store.seg.durable()} of "
                                   f"{self.store.seg.last_token}, store {self.store.seg.stats()})")
            t0 = _time.monotonic()
            if self.pending:
                self.store.seg.wait(self.pending[0].token, 1.0)
            else:
                _time.sleep(0.001)              # only the topic holds buffers: wait for its retention
            self.disk_wait_s += _time.monotonic() - t0

    def publish(self, b: _BlockBuf, nbytes: int, first_seq: int, now_ms: int, tag=None) -> int:
        """The block is in ``b``: zero its padding, seal it, queue it to the store, publish it."""
        nbytes = int(nbytes)
        pad = -(-nbytes // SEG_ALIGN) * SEG_ALIGN
        if pad > nbytes:
            ctypes.memset(b.host + nbytes, 0, pad - nbytes)
        native().swseg_seal(b.host, int(first_seq), int(now_ms), self.boot, self.rank, self.world)
        n_rows = int(np.frombuffer((ctypes.c_uint8 * 64).from_address(b.host), np.uint8).view(HDR)[0]["n_rows"])
        toff = int(native().swseg_ix_offset(b.host))
        if toff:
            self.index_bytes += nbytes - toff           # the block's index trailer (swindex.h)
        with self._lock:
            b.refs += 1                                    # the store's reference
        tok = self.store.add_block(b.host, nbytes, owner=b)
        if tok < 0:                     # a replayed block the store already holds
            self._release(b)
            self.tags.append((self.store.seg.last_token, tag))   # durable with everything before it
        else:
            b.token = tok
            self.pending.append(b)
            self.tags.append((tok, tag))
        if self.bus is not None and self.topic is not None:
            with self._lock:
                b.refs += 1                                # the topic's reference
            self.bus.append_external(self.topic, self.partition, b, b.host, nbytes, ts=int(now_ms),
                                     on_release=self._release)
        self._release(b)                                   # the copy's reference
        self.blocks += 1
        self.bytes += nbytes
        self.rows += n_rows
        return tok

    def committable(self) -> list:
        """Tags of the blocks that are durable now (removed from the pending list)."""
        d = self.store.durable()
        out = []
        while self.tags and self.tags[0][0] <= d:
            out.append(self.tags.pop(0)[1])
        return out

    def flush(self, timeout_s: float = 120.0) -> bool:
        ok = self.store.flush(timeout_s)
        self._reap()
        return ok


_ETYPE = {DeviceEventType.Measurement: EV_MEASUREMENT, DeviceEventType.Location: EV_LOCATION,
          DeviceEventType.Alert: EV_ALERT, DeviceEventType.StateChange: EV_STATE_CHANGE,
          DeviceEventType.CommandInvocation: EV_COMMAND_INVOCATION,
          DeviceEventType.CommandResponse: EV_COMMAND_RESPONSE}
_LEVELS = [AlertLevel.Info, AlertLevel.Warning, AlertLevel.Error, AlertLevel.Critical]
_CTX = {DeviceEventIndex.Assignment: 0, DeviceEventIndex.Customer: 2, DeviceEventIndex.Area: 3,
        DeviceEventIndex.Asset: 4}


def boot_id(boot) -> int:
    """Numeric engine incarnation of a tenant's boot string (hex ms timestamp) or number."""
    return int(boot, 16) if isinstance(boot, str) else int(boot or 0)


def _leased(fn):
    """Run a read method under a segment-store read lease (re-entrant per thread): the in-memory
    trailer and block copies it reaches stay valid until it returns."""
    @functools.wraps(fn)
    def run(self, *a, **k):
        if getattr(self._tl, "leased", False):
            return fn(self, *a, **k)
        self._tl.leased = True
        try:
            with self.seg.lease():
                return fn(self, *a, **k)
        finally:
            self._tl.leased = False
    return run


class _FileMap:
    """A read-only shared map of a segment file (libc ``mmap``: it may reserve more than the file
    holds, which Python's ``mmap`` refuses), unmapped when the last holder lets go."""

    _libc = None

    def __init__(self, fd: int, length: int):
        if _FileMap._libc is None:
            lib = ctypes.CDLL(None, use_errno=True)
            lib.mmap.restype = ctypes.c_void_p
            lib.mmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_long]
            lib.munmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
            _FileMap._libc = lib
        self.length = int(length)
        a = _FileMap._libc.mmap(None, self.length, 1, 1, int(fd), 0)      # PROT_READ, MAP_SHARED
        self.addr = 0 if a in (None, ctypes.c_void_p(-1).value) else int(a)

    def __del__(self):
        if self.addr and _FileMap._libc is not None:
            _FileMap._libc.munmap(self.addr, self.length)
            self.addr = 0


class DurableEventStore(DeviceEventStore):
    """Event store of engine tenants on durable segments (see module docstring).

    Ingest: :meth:`add_block` (an encoded, sealed block + the dictionary deltas its rows need).
    Events are identified by (boot, rank, store sequence): a block whose rows the store already
    holds for its (boot, rank) is skipped (a shard replaying after a restore).  Assignment and name
    indices are engine-local, so the dictionaries are kept per boot; their deltas are fsync'd to
    ``dict-<rank>.log`` before the block is queued, so a durable block never refers to an unknown
    entry."""

    def __init__(self, directory: str, rank: int = 0, rotate_bytes: int = 1 << 30, retention_bytes: int = 0,
                 direct: bool = True, cache_blocks: int = 8, index: bool = True, index_threads: int | None = None,
                 block_cache_bytes: int | None = None):
        # (index / index_threads: accepted for callers of the host indexer this store no longer needs --
        # every block arrives with its index trailer)
        self.dir = directory
        os.makedirs(directory, exist_ok=True)
        self.rotate_bytes = int(rotate_bytes)
        self.seg = SegmentStore(directory, rank, rotate_bytes, retention_bytes, direct)
        # the scan images of recent blocks (page headers + leading columns) kept in memory as the
        # blocks are written (the writes bypass the page cache): listings over fresh data -- the
        # usual page-1 query -- do not wait on the device
        if block_cache_bytes is None:
            # ~6 B per stored event: sized to hold the whole retained store's images where the host
            # has the memory (an eighth of it, at most 32 GB)
            env = os.environ.get("SW_STORE_SCAN_CACHE_GB")
            if env is not None:
                block_cache_bytes = int(float(env) * (1 << 30))
            else:
                try:
                    ram = os.sysconf("SC_PAGE_SIZE") * os.sysconf("SC_PHYS_PAGES")
                except (ValueError, OSError, AttributeError):
                    ram = 32 << 30
                block_cache_bytes = int(min(32 << 30, ram // 8))
        self.seg.mem_caps(-1, int(block_cache_bytes))
        self._tl = threading.local()
        self._asg: dict[int, dict[int, list]] = {}       # boot -> assignment index -> [asg, dev, cust, area, asset]
        self._names: dict[int, dict[int, str]] = {}      # boot -> name id -> name
        self._ctx: dict[int, dict[int, dict]] = {}       # boot -> dimension -> context token -> engine id
        self._dict_version = 0
        self._ctx_arr: dict[int, np.ndarray] = {}          # boot -> [3, cap] context id by assignment index
        self._asg_n: dict[int, int] = {}                   # boot -> max assignment index + 1
        self._asg_tok: dict[int, dict[str, list]] = {}     # boot -> assignment token -> assignment indexes
        self._rules: dict[str, str] = {}                 # alert type -> rule message
        self._lock = threading.RLock()
        self._dict_path = os.path.join(directory, f"dict-{rank}.log")
        self._load_dict()
        self._dict_f = open(self._dict_path, "ab")
        self._high: dict[tuple, int] = {}
        self._pending_ends: dict[tuple, list] = {}       # (boot, rank) -> [(sequence end, token)] queued
        for e in self.seg.index():
            key = (int(e["boot"]), int(e["rank"]))
            self._high[key] = max(self._high.get(key, 0), int(e["first_seq"]) + int(e["n_rows"]))
        self._cache: OrderedDict = OrderedDict()       # block key -> decoded columns
        self.cache_blocks = cache_blocks
        self._pages: OrderedDict = OrderedDict()       # (block key, page) -> decoded page columns
        self.cache_pages = 256
        self.skipped_rows = 0
        # every block carries its index trailer (swindex.h, built with the block): memory maps of
        # the trailers (LRU), the per-boot tables of trailer addresses for the native reads
        self._tmaps: OrderedDict = OrderedDict()
        self.max_maps = 16384
        self._tabs = None
        self.scan_threads = int(os.environ.get("SW_STORE_SCAN_THREADS", "16"))
        # events added through the API (REST / RPC adds, command invocations and responses, rule
        # alerts): rows of blocks like the engine's (api_blocks.py).  Until a block holds them they
        # are the tail: in memory and in a short checksummed log, fdatasync'd before the add returns
        self.api_flush_events = int(os.environ.get("SW_API_FLUSH_EVENTS", 65536))
        self.api_flush_s = float(os.environ.get("SW_API_FLUSH_S", 1.0))
        self._api_lock = threading.Lock()
        self._api_flush_mu = threading.Lock()
        self._api_boot = self._load_api_boot(directory, rank)
        self._api_next = self._high.get((self._api_boot, 0), 0)
        self._api_tail: list = []                         # (sequence, event), in sequence order
        self._objects = MemoryEventStore()                # the tail's events, indexed
        self._api_dic = None
        self._api_path = os.path.join(directory, f"api-{rank}.log")
        self._load_api_log()
        self._api_f = open(self._api_path, "ab")
        self._api_stop = threading.Event()
        self._api_kick = threading.Event()
        self._api_err: str | None = None
        self._api_th = threading.Thread(target=self._api_flush_loop, name="api-blocks", daemon=True)
        self._api_th.start()

    # ------------------------------------------------------------------ API-added events
    @staticmethod
    def _load_api_boot(directory: str, rank: int) -> int:
        """The store's API boot: the engine-incarnation id API-added events are stored under, fixed
        for the directory (so their ids and dictionaries continue across restarts).  Bit 52 keeps it
        apart from engine boots (millisecond timestamps)."""
        path = os.path.join(directory, f"api-boot-{rank}")
        try:
            with open(path) as f:
                return int(f.read().strip(), 16)
        except (OSError, ValueError):
            pass
        boot = (1 << 52) | int(time.time() * 1000)
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            f.write(f"{boot:x}\n")
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, path)
        return boot

    def _load_api_log(self):
        """Replay ``api-<rank>.log`` (``<crc32 hex> {"s": sequence, "e": event}`` per line): events a
        block already holds are skipped, the rest are the tail.  A torn or corrupt tail (a crash
        mid-write: the add never returned) is cut off; lines of older logs without a sequence get one."""
        if not os.path.exists(self._api_path):
            return
        good, tail, renumbered = 0, [], False
        covered = self._high.get((self._api_boot, 0), 0)
        with open(self._api_path, "rb") as f:
            for line in f:
                if not line.endswith(b"\n") or len(line) < 10 or line[8:9] != b" ":
                    break
                body = line[9:-1]
                try:
                    if int(line[:8], 16) != zlib.crc32(body):
                        break
                    d = json.loads(body)
                    if "s" in d and "e" in d:
                        seq, ev = int(d["s"]), event_from_dict(d["e"])
                    else:                                  # a line of an older log: no sequence yet
                        seq, ev, renumbered = -1, event_from_dict(d), True
                except (ValueError, KeyError, TypeError):
                    break
                good += len(line)
                if seq < 0:
                    seq = max(self._api_next, covered)
                    ev.id = f"{self._api_boot:x}-{seq}"
                if seq >= covered:
                    tail.append((seq, ev))
                self._api_next = max(self._api_next, seq + 1, covered)
        tail.sort(key=lambda x: x[0])
        self._api_tail = tail
        self._objects.add_events([e for _, e in tail])
        if good < os.path.getsize(self._api_path) or renumbered or len(tail) == 0:
            self._rewrite_api_log(tail)

    @staticmethod
    def _api_line(seq: int, e) -> bytes:
        body = json.dumps({"s": seq, "e": e.to_dict()}, separators=(",", ":")).encode()
        return b"%08x %s\n" % (zlib.crc32(body), body)

    def _rewrite_api_log(self, tail):
        """Replace the log by the tail's lines (a new file, fsync'd, renamed over the old one)."""
        tmp = self._api_path + ".tmp"
        with open(tmp, "wb") as f:
            f.write(b"".join(self._api_line(s_, e) for s_, e in tail))
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, self._api_path)
        dfd = os.open(os.path.dirname(os.path.abspath(self._api_path)), os.O_RDONLY)
        try:
            os.fsync(dfd)
        finally:
            os.close(dfd)

    def add_events(self, events):
        """Durable API add: the store gives each event its id (``<api boot hex>-<sequence>``), the
        events are on disk (one fdatasync per call) and visible before the call returns; a block
        holds them once the tail is flushed (see api_blocks.py)."""
        if not events:
            return events
        from .api_blocks import row_limit_error
        for e in events:                 # refused before the log: a row no block can hold
            why = row_limit_error(e)
            if why is not None:
                from ..core.errors import ErrorCode, SiteWhereSystemException
                raise SiteWhereSystemException(ErrorCode.Error, detail=f"event not stored: {why}")
        now = int(time.time() * 1000)
        with self._api_lock:
            lines = []
            for e in events:
                seq = self._api_next
                self._api_next += 1
                e.id = f"{self._api_boot:x}-{seq}"
                if e.received_date is None:
                    e.received_date = now
                lines.append(self._api_line(seq, e))
                self._api_tail.append((seq, e))
            self._api_f.write(b"".join(lines))
            self._api_f.flush()
            os.fdatasync(self._api_f.fileno())
            self._objects.add_events(events)
            if len(self._api_tail) >= self.api_flush_events:
                self._api_kick.set()
        return events

    def _api_flush_loop(self):
        while not self._api_stop.is_set():
            self._api_kick.wait(self.api_flush_s)
            self._api_kick.clear()
            if self._api_stop.is_set():
                break
            try:
                self.flush_api()
                self._api_err = None
            except Exception as e:  # noqa: BLE001 -- the tail stays in the log; retried next round
                self._api_err = f"{type(e).__name__}: {e}"
                import logging
                logging.getLogger(__name__).error("API event tail flush failed (retried): %s", self._api_err)

    def _api_dictionary(self):
        from .api_blocks import ApiDictionary
        if self._api_dic is None:
            b = self._api_boot
            with self._lock:
                self._api_dic = ApiDictionary(self._asg.get(b, {}), self._names.get(b, {}),
                                              {d: dict(m) for d, m in self._ctx.get(b, {}).items()})
        return self._api_dic

    def flush_api(self, max_rows: int = 1 << 20) -> int:
        """Encode the tail into blocks (index trailers included), make them durable, then cut the
        tail and the log back to what came after.  Returns the events flushed."""
        from .api_blocks import encode_events
        with self._api_flush_mu:
            with self._api_lock:
                batch = list(self._api_tail)
            if not batch:
                return 0
            dic = self._api_dictionary()
            for i in range(0, len(batch), max_rows):
                chunk = batch[i:i + max_rows]
                evs = [e for _, e in chunk]
                rows, recs, spans, raw = encode_events(evs, dic)
                blk = encode_block(rows, recs, spans, raw, index=True, ctx=dic.ctx_table())
                recv = max(int(e.received_date or 0) for e in evs)
                seal(blk, chunk[0][0], recv, self._api_boot, 0, 1)
                d_asg, d_names, d_ctx = dic.take_delta()
                tok = self.add_block(_p(blk), len(blk), blk, boot=self._api_boot, asg=d_asg, names=d_names,
                                     ctx=d_ctx)
                if tok >= 0 and not self.wait(tok):
                    raise TimeoutError("API event block not durable in time")
            upto = batch[-1][0] + 1
            with self._api_lock:
                rest = [(s_, e) for s_, e in self._api_tail if s_ >= upto]
                objs = MemoryEventStore()
                objs.add_events([e for _, e in rest])
                self._api_tail, self._objects = rest, objs
                self._api_f.close()
                self._rewrite_api_log(rest)
                self._api_f = open(self._api_path, "ab")
            return len(batch)

    def _api_covered(self, tabs) -> int:
        """The API boot's sequences that blocks in ``tabs`` hold (events below it left the tail)."""
        t = tabs.get(self._api_boot)
        if t is None or not t["n"]:
            return 0
        return int((t["ents"]["first_seq"].astype(np.int64) + t["ents"]["n_rows"].astype(np.int64)).max())

    def _api_seq(self, ev) -> int:
        b, _, n = (ev.id or "").rpartition("-")
        try:
            return int(n) if int(b, 16) == self._api_boot else -1
        except ValueError:
            return -1

    # ------------------------------------------------------------------ dictionaries
    def _load_dict(self):
        if not os.path.exists(self._dict_path):
            return
        with open(self._dict_path, "rb") as f:
            for line in f:
                try:
                    d = json.loads(line)
                except ValueError:
                    break                                  # torn last line
                self._apply_dict(d)

    def _apply_dict(self, d: dict):
        """Apply a dictionary delta, keeping the reverse maps the read path uses current in O(delta):
        assignment token -> indexes, and the context id of every assignment per dimension (rebuilt in
        full only when new context tokens arrive -- new customers / areas / assets, not new rows)."""
        b = int(d.get("boot", 0))
        asg = self._asg.setdefault(b, {})
        tok = self._asg_tok.setdefault(b, {})
        delta = {int(k): v for k, v in (d.get("asg") or {}).items()}
        for k, v in delta.items():
            old = asg.get(k)
            if old and old[0] != v[0] and k in tok.get(old[0], ()):
                tok[old[0]].remove(k)
            if not old or old[0] != v[0]:
                tok.setdefault(v[0], []).append(k)
        asg.update(delta)
        self._names.setdefault(b, {}).update({int(k): v for k, v in (d.get("names") or {}).items()})
        self._rules.update(d.get("rules") or {})
        new_ctx = False
        for dim, m in (d.get("ctx") or {}).items():
            self._ctx.setdefault(b, {}).setdefault(int(dim), {}).update({str(k): int(v) for k, v in m.items()})
            new_ctx = True
        if delta:
            self._asg_n[b] = max(self._asg_n.get(b, 0), max(delta) + 1)
        if new_ctx:
            self._ctx_fill(b, asg.items())
        elif delta and b in self._ctx_arr:
            self._ctx_fill(b, delta.items())
        self._dict_version += 1

    def _ctx_fill(self, b: int, items):
        """Context ids (customer, area, asset) of the given assignment entries into the boot's table."""
        ids = self._ctx.get(b)
        if not ids:
            return
        n = self._asg_n.get(b, 0)
        arr = self._ctx_arr.get(b)
        if arr is None or arr.shape[1] < n:
            grown = np.full((3, max(1024, n, 2 * (0 if arr is None else arr.shape[1]))), -1, np.int32)
            if arr is not None:
                grown[:, :arr.shape[1]] = arr
            else:
                items = self._asg.get(b, {}).items()       # a new table holds every known assignment
            arr = grown
        dims = [ids.get(dd, {}) for dd in range(3)]
        for k, v in items:
            for dd in range(3):
                arr[dd, k] = dims[dd].get(v[2 + dd], -1) if len(v) > 2 + dd else -1
        self._ctx_arr[b] = arr

    def add_dictionary(self, boot, asg: dict | None = None, names: dict | None = None, rules: dict | None = None,
                       ctx: dict | None = None):
        """Dictionary deltas of an engine incarnation: assignment index -> [assignment, device,
        customer, area, asset, ...], name id -> name, rule alert type -> message, and ``ctx`` =
        {dimension (0 customer, 1 area, 2 asset): {context token: engine id}} -- the ids the block
        index trailers key their context dimensions by."""
        b = boot_id(boot)
        d = {"boot": b}
        if asg:
            d["asg"] = {int(k): list(v) for k, v in asg.items()}
        if names:
            d["names"] = {int(k): v for k, v in names.items()}
        if ctx:
            cur = self._ctx.get(b, {})
            delta = {str(int(dim)): {str(k): int(v) for k, v in m.items() if cur.get(int(dim), {}).get(str(k)) != int(v)}
                     for dim, m in ctx.items()}
            delta = {k: v for k, v in delta.items() if v}
            if delta:
                d["ctx"] = delta
        if rules and any(self._rules.get(k) != v for k, v in rules.items()):
            d["rules"] = dict(rules)
        if len(d) == 1:
            return
        with self._lock:
            self._apply_dict(d)
            self._dict_f.write((json.dumps(d, separators=(",", ":")) + "\n").encode())
            self._dict_f.flush()
            os.fdatasync(self._dict_f.fileno())

    # ------------------------------------------------------------------ ingest
    def add_block(self, ptr: int, nbytes: int, owner=None, boot=None, asg=None, names=None, rules=None,
                  src=None, ctx=None) -> int:
        """Queue a sealed block for the disk; returns its token.  A replay of rows already queued
        returns the token of the block holding them (-1 once they are durable).
        ``src``: input offsets the block completes (see :meth:`SegmentStore.append`; the block must
        carry ``FLAG_COMMIT``)."""
        h = np.frombuffer((ctypes.c_uint8 * 64).from_address(ptr), np.uint8).view(HDR)[0]
        b = int(h["boot"])
        if boot is not None and boot_id(boot) != b:
            raise ValueError("dictionary boot differs from the block's")
        self.add_dictionary(b, asg, names, rules, ctx)
        key, first, n = (b, int(h["rank"])), int(h["first_seq"]), int(h["n_rows"])
        if src is not None and not int(h["flags"]) & FLAG_COMMIT:
            raise ValueError("a block with input offsets must be sealed with FLAG_COMMIT")
        with self._lock:
            if n and first + n <= self._high.get(key, 0):
                # a replay of rows already queued: it is "stored" only once those rows are durable --
                # hand back the token that makes them so (a failed write raises here, never skips)
                self.seg.durable()
                tok = self._covering_token(key, first + n)
                self.skipped_rows += n
                return tok
            # the high-water mark moves only once the block is queued: a failed append leaves it, so
            # the retried batch is written instead of skipped as a replay
            tok = self.seg.append(ptr, nbytes, owner, src)
            self._high[key] = max(self._high.get(key, 0), first + n)
            self._pending_ends.setdefault(key, []).append((first + n, tok))
            return tok

    def _covering_token(self, key, end: int) -> int:
        """Token of the earliest queued block of ``key`` reaching ``end`` that is not durable yet;
        -1 when every such block is on disk."""
        d = self.seg.durable()
        ends = [e for e in self._pending_ends.get(key, []) if e[1] > d]
        self._pending_ends[key] = ends
        for e, tok in ends:
            if e >= end:
                return tok
        return -1

    def source_offset(self, topic: str, partition: int) -> int | None:
        """Next input offset of (topic, partition) whose events are all durable here (None: none
        recorded).  A restarted tenant resumes there: nothing lost, nothing stored twice."""
        return self.seg.source_offset(topic, partition)

    def add_encoded(self, block: np.ndarray, **dicts) -> int:
        return self.add_block(_p(block), len(block), block, **dicts)

    def durable(self) -> int:
        return self.seg.durable()

    def wait(self, token: int, timeout_s: float = 60.0) -> bool:
        return self.seg.wait(token, timeout_s)

    def flush(self, timeout_s: float = 60.0) -> bool:
        return self.seg.flush(timeout_s)

    def close(self):
        self._api_stop.set()
        self._api_kick.set()
        self._api_th.join(timeout=30)
        try:
            self.flush_api()                           # the tail into a block: a short restart
        except Exception:  # noqa: BLE001 -- it stays in the log
            pass
        self._tabs = None
        self._tmaps.clear()
        self.seg.close()
        for f in (self._dict_f, self._api_f):
            try:
                f.close()
            except Exception:  # noqa: BLE001
                pass

    # ------------------------------------------------------------------ block index trailers
    @staticmethod
    def _key(ent) -> tuple:
        """A block's identity across processes and reopen (segment file ids are per process)."""
        return int(ent["boot"]), int(ent["rank"]), int(ent["first_seq"]), int(ent["n_rows"])

    def _trailer(self, ent):
        """(address, bytes, header) of a block's index trailer, memory-mapped from its segment file
        (read-only; the page cache keeps the hot ones), or None for a block without one.  The store
        verified the trailer when it recovered the block on open or wrote it itself."""
        key = self._key(ent)
        with self._lock:
            m = self._tmaps.get(key)
            if m is not None:
                self._tmaps.move_to_end(key)
                return m[0]
        path = self.seg.file_path(int(ent["file"]))
        if path is None:
            return None
        off, nb = int(ent["offset"]), int(ent["bytes"])
        import mmap as _mmap
        fd = os.open(path, os.O_RDONLY)
        try:
            h = np.frombuffer(os.pread(fd, 64, off), HDR)[0]
            if not int(h["flags"]) & FLAG_INDEX:
                res = None
                mm = None
            else:
                npg = int(h["n_pages"])
                tstart = int(np.frombuffer(os.pread(fd, 4, off + 64 + 4 * npg), np.uint32)[0])
                t0 = off + tstart
                a0 = t0 & ~(_mmap.ALLOCATIONGRANULARITY - 1)
                mm = _mmap.mmap(fd, off + nb - a0, prot=_mmap.PROT_READ, offset=a0)
                arr = np.frombuffer(mm, np.uint8)
                view = arr[t0 - a0:]
                th = view[:128].view(IX_HDR)[0]
                if int(th["magic"]) != IX_MAGIC or int(th["bytes"]) != nb - tstart or \
                        int(th["n_rows"]) != int(h["n_rows"]):
                    raise ValueError("block index trailer does not match its block")
                res = (view.ctypes.data, int(th["bytes"]), th, view)
        finally:
            os.close(fd)
        with self._lock:
            self._tmaps[key] = (res, mm)
            while len(self._tmaps) > self.max_maps:
                self._tmaps.popitem(last=False)
        return res

    @staticmethod
    def _trailer_mem(addr: int, nbytes: int, ent):
        """(address, bytes, header, view) of a trailer copy the segment store holds in memory."""
        view = np.ctypeslib.as_array((ctypes.c_uint8 * int(nbytes)).from_address(int(addr)))
        th = view[:128].view(IX_HDR)[0]
        if int(th["magic"]) != IX_MAGIC or int(th["bytes"]) != int(nbytes) or int(th["n_rows"]) != int(ent["n_rows"]):
            raise ValueError("block index trailer does not match its block")
        return (int(addr), int(nbytes), th, view)

    def _boot_tables(self) -> dict:
        """Per boot: the blocks (store order) and their trailer addresses (0: none) for the native
        multi-block reads.  Trailers come from the segment store's in-memory copies (made while
        each block was written), else memory-mapped from the files.  Kept across appends: only
        new blocks (and blocks whose copy changed) are resolved."""
        ents, taddr, tlen, baddr = self.seg.index_tr()
        ver = (len(ents), int(ents["first_seq"][-1]) if len(ents) else 0, int(ents["first_seq"][0]) if len(ents) else 0)
        tabs = self._tabs
        if tabs is not None and tabs[0] == ver and np.array_equal(tabs[2], taddr) and np.array_equal(tabs[3], baddr):
            return tabs[1]
        res = {}
        P = ctypes.c_void_p
        prev = tabs[1] if tabs is not None else {}
        boots = ents["boot"].astype(np.int64)
        removed = False
        for b in dict.fromkeys(boots.tolist()):
            m = boots == b
            lst, ta, tl, ba = ents[m], taddr[m], tlen[m], baddr[m]
            old = prev.get(b)
            k, j = 0, 0
            if old is not None and old["n"] and len(lst):
                # appends, and retention dropping the oldest files (the steady state of a store
                # bounded by rows: both at once, every few commits): keep the blocks already resolved
                # -- the old list's blocks from the new first one on, if they are the new list's prefix
                of, orank = old["ents"]["first_seq"], old["ents"]["rank"]
                hit = np.nonzero((of == lst["first_seq"][0]) & (orank == lst["rank"][0]))[0]
                if len(hit):
                    j = int(hit[0])
                    k = old["n"] - j
                    if k > len(lst) or not (np.array_equal(of[j:], lst["first_seq"][:k])
                                            and np.array_equal(orank[j:], lst["rank"][:k])):
                        k, j = 0, 0
            removed |= old is not None and (j > 0 or k < old["n"])
            trs = list(old["tr"][j:j + k]) if k else []
            for i in np.nonzero(ta[:k] != old["taddr"][j:j + k])[0].tolist() if k else []:
                trs[i] = self._trailer_mem(ta[i], tl[i], lst[i]) if ta[i] else self._trailer(lst[i])
            trs += [self._trailer_mem(ta[i], tl[i], lst[i]) if ta[i] else self._trailer(lst[i])
                    for i in range(k, len(lst))]
            addrs = [t[0] if t is not None else 0 for t in trs]
            res[b] = {"ents": lst, "tr": trs, "n": len(lst), "addr": (P * len(lst))(*addrs), "taddr": ta, "baddr": ba,
                      "first": lst["first_seq"].astype(np.int64), "world": lst["world"].astype(np.int64),
                      "rank": lst["rank"].astype(np.int64)}
        if removed or len(prev) > len(res):
            live = {self._key(e) for e in ents}
            with self._lock:
                for k in [k for k in self._tmaps if k not in live]:      # retention removed the block
                    self._tmaps.pop(k, None)
        self._tabs = (ver, res, taddr, baddr)
        return res

    def retention_state(self) -> dict:
        """Retention limits and what the store holds (rows / bytes retained and deleted), plus the
        API tail's flush health (``api_flush_error``: the last failed flush, None when healthy)."""
        st = self.seg.stats()
        return {k: st[k] for k in ("retention_rows", "retention_bytes", "retained_rows", "retained_bytes",
                                   "deleted_rows", "deleted_bytes", "deleted_files", "files")} | {
            "api_tail": len(self._api_tail), "api_flush_error": self._api_err, "rotate_bytes": self.rotate_bytes}

    # the fewest bytes a stored row takes (a block's columns + index run 14-19 B per row)
    MIN_ROW_BYTES = 8

    def limit_retention_rows(self, rows: int) -> int:
        """Keep at most ``rows`` event rows (whole segment files, oldest first, checked after every
        group commit): an engine tenant whose store-backed dedup filter remembers its newest N ids sets
        this, so the store holds no id the filter has forgotten.  New files then start small enough
        to hold at most a quarter of the limit, so the file being written (never deleted) keeps the
        store within 1.25x of it, and what the limit deletes comes back in quarter steps.  Only ever
        tightens.  Returns the limit in force."""
        cur = self.seg.stats()["retention_rows"]
        rows = int(rows)
        if rows > 0 and (cur <= 0 or rows < cur):
            rotate = min(self.rotate_bytes, max(1 << 20, rows * self.MIN_ROW_BYTES // 4)) >> 12 << 12
            self.seg.set_retention(0, rows, rotate)
            self.rotate_bytes = rotate
            cur = rows
        return cur

    def index_wait(self, timeout_s: float = 60.0) -> bool:
        """Every block is indexed as it is written (its trailer): nothing to wait for."""
        return True

    @_leased
    def index_stats(self) -> dict:
        tabs = self._boot_tables()
        n = sum(t["n"] for t in tabs.values())
        ix = [tr for t in tabs.values() for tr in t["tr"] if tr is not None]
        return {"blocks": n, "indexed": len(ix), "index_bytes": sum(tr[1] for tr in ix)}

    @_leased
    def alternate_id_count(self) -> int:
        """Alternate ids stored (every block's trailer count; blocks without a trailer decoded)."""
        total = 0
        for t in self._boot_tables().values():
            for e, tr in zip(t["ents"], t["tr"]):
                total += int(tr[2]["n_alt"]) if tr is not None else len(self._block_alt_hashes(e))
        return total

    def _block_alt_hashes(self, ent) -> np.ndarray:
        blk = self.seg.read_block(ent)
        out = np.empty(int(ent["n_rows"]), np.uint64)
        n = int(native().swseg_alt_hashes(_p(blk), _p(out), len(out)))
        if n < 0:
            raise ValueError("event block decode failed")
        return out[:n]

    def alternate_hash_chunks(self, max_ids: int = 1 << 26, wait_s: float = 0.0, threads: int = 16, skip: int = 0):
        """The stored alternate-id hashes, newest blocks first, one numpy u64 chunk per block, at most
        ``max_ids`` after the first ``skip`` of that order: what a restarted engine seeds its
        store-backed dedup filter with.  The trailers keep only fingerprints, so the blocks' id
        columns are decoded (natively, on ``threads`` threads; ctypes releases the interpreter
        meanwhile); skipped blocks are counted from their trailers, not decoded."""
        from concurrent.futures import ThreadPoolExecutor
        with self.seg.lease():            # the trailers' id counts, read while they are held
            pairs = [(e, int(tr[2]["n_alt"]) if tr is not None else None)
                     for t in self._boot_tables().values() for e, tr in zip(t["ents"], t["tr"])]
        pairs.sort(key=lambda x: (int(x[0]["recv_ms"]), int(x[0]["first_seq"])), reverse=True)
        ents = []
        for e, n in pairs:
            # whole blocks are skipped by their trailer counts only up to the first block kept: the
            # rest of the skip (if any) is cut from the decoded ids below, in order
            if not ents and skip > 0 and n is not None and skip >= n:
                skip -= n
                continue
            ents.append(e)
        left = int(max_ids) + int(skip)
        with ThreadPoolExecutor(max(1, threads)) as pool:
            for i in range(0, len(ents), max(1, threads)):
                if left <= 0:
                    break
                for h in pool.map(self._block_alt_hashes, ents[i:i + threads]):
                    if left <= 0:
                        break
                    take = h[:left]
                    left -= len(take)
                    if skip:
                        cut = min(skip, len(take))
                        take, skip = take[cut:], skip - cut
                    if len(take):
                        yield take

    def _alt_candidates(self, hashes) -> dict:
        """hash -> [(boot table, block position, page)] of the blocks whose trailer holds a fingerprint
        match, newest block first (native, over every block of every boot per hash)."""
        lib = native()
        out: dict = {}
        cap = 256
        bo, po = np.empty(cap, np.int64), np.empty(cap, np.int64)
        for b, t in self._boot_tables().items():
            for hv in hashes:
                k = int(lib.swseg_ix_alt_pages(t["addr"], t["n"], int(hv), _p(bo), _p(po), cap))
                for j in range(min(k, cap)):
                    out.setdefault(int(hv), []).append((t, int(bo[j]), int(po[j])))
        return out

    @_leased
    def find_alternate_hashes(self, hashes, covered: tuple | None = None, indexed_only: bool = False) -> dict:
        """alt-id hash -> event id string for the hashes stored on disk, the newest event per hash
        (store-backed dedup beyond the engine's window: ``AlternateIdDeduplicator`` asks the event
        store whether the id was ever seen).  Every block's trailer is searched natively; a
        fingerprint hit is confirmed on its page (the full 64-bit hash of the stored id string).
        ``covered`` / ``indexed_only``: kept for callers; blocks without a trailer (older stores) are
        scanned unless ``indexed_only``."""
        want = [int(h) for h in np.unique(np.asarray(list(hashes), np.uint64))]
        found: dict = {}
        if not want:
            return found
        cands = self._alt_candidates(want)
        by_tab: dict = {}
        for hv, lst in cands.items():
            for t, bi, page in lst:
                by_tab.setdefault(id(t), (t, []))[1].append((bi, page, hv))
        best: dict = {}                               # hash -> (recv_ms, block position, row, boot table)
        for t, lst in by_tab.values():
            bis = np.array([x[0] for x in lst], np.int64)
            ci, rows = self._alt_page_rows(t, bis, [x[1] for x in lst], [x[2] for x in lst])
            for c, r in zip(ci.tolist(), rows.tolist()):
                hv = lst[c][2]
                bi = lst[c][0]
                key = (int(t["ents"][bi]["recv_ms"]), bi, r)
                if hv not in best or key > best[hv][0]:
                    best[hv] = (key, t, bi, r)
        for hv, (_, t, bi, r) in best.items():
            e = t["ents"][bi]
            found[hv] = f"{int(e['boot']):x}-{int(self._eids(e, [r])[0])}"
        if not indexed_only:
            for t in self._boot_tables().values():
                for e, tr in zip(t["ents"], t["tr"]):
                    if tr is not None:
                        continue
                    if covered is not None and int(e["boot"]) == covered[0] and int(e["rank"]) == covered[1] \
                            and int(e["first_seq"]) >= covered[2]:
                        continue
                    cols = self._decoded(e)
                    for i in range(len(cols["date"]) - 1, -1, -1):
                        if not int(cols["flags"][i]) & SEGF_HAS_ALT:
                            continue
                        from ..pipeline.fleet import hash64
                        hv = hash64(row_strings(cols, i)[0])
                        if hv in want and hv not in found:
                            found[hv] = f"{int(e['boot']):x}-{int(self._eids(e, [i])[0])}"
        return found

    @_leased
    def get_event_by_alternate_id(self, alt: str):
        from ..pipeline.fleet import hash64
        ev = self._objects.get_event_by_alternate_id(alt)
        if ev is not None:
            return ev
        h = hash64(alt)
        lst = self._alt_candidates([h]).get(h, [])
        by_tab: dict = {}
        for t, bi, page in lst:
            by_tab.setdefault(id(t), (t, []))[1].append((bi, page))
        hits = []                                     # (recv_ms, block position, row, boot table)
        for t, cl in by_tab.values():
            bis = np.array([x[0] for x in cl], np.int64)
            ci, rows = self._alt_page_rows(t, bis, [x[1] for x in cl], [h] * len(cl))
            hits += [(int(t["ents"][bis[c]]["recv_ms"]), int(bis[c]), int(r), t) for c, r in zip(ci.tolist(), rows.tolist())]
        hits.sort(key=lambda x: x[:3], reverse=True)
        for _, bi, r, t in hits:                      # newest first; the id string settles a hash collision
            cols = self._fetch(t, [bi], [r])
            if row_strings(cols, 0)[0] == alt:
                return self._materialize(cols, 0)
        for t in self._boot_tables().values():                 # blocks without a trailer
            for e, tr in zip(t["ents"][::-1], t["tr"][::-1]):
                if tr is not None:
                    continue
                cols = self._decoded(e)
                for i in range(len(cols["date"]) - 1, -1, -1):
                    if int(cols["flags"][i]) & SEGF_HAS_ALT and row_strings(cols, i)[0] == alt:
                        return self._materialize(cols, i)
        return None

    # ------------------------------------------------------------------ page reads
    def _read_pages(self, ent, p0: int, p1: int) -> np.ndarray:
        """A block buffer holding only its header, page table and pages [p0, p1) (checked), read
        with three preads: a point query touches a few KB of a block, not the whole block."""
        path = self.seg.file_path(int(ent["file"]))
        if path is None:
            raise KeyError("segment file deleted by retention")
        off = int(ent["offset"])
        fd = os.open(path, os.O_RDONLY)
        try:
            head = os.pread(fd, 64, off)
            h = np.frombuffer(head, HDR)[0]
            tbl_len = -(-4 * (int(h["n_pages"]) + 1) // 8) * 8
            tbl = os.pread(fd, tbl_len, off + 64)
            pt = np.frombuffer(tbl, np.uint32)
            lo, hi = int(pt[p0]), int(pt[p1])
            buf = np.empty(int(h["bytes"]), np.uint8)
            buf[:64] = np.frombuffer(head, np.uint8)
            buf[64:64 + tbl_len] = np.frombuffer(tbl, np.uint8)
            buf[lo:hi] = np.frombuffer(os.pread(fd, hi - lo, off + lo), np.uint8)
        finally:
            os.close(fd)
        rc = int(native().swseg_verify_pages(_p(buf), len(buf), int(p0), int(p1)))
        if rc:
            raise ValueError(f"corrupt event block (code {rc})")
        return buf

    def _page_cols(self, ent, page: int) -> dict:
        """Decoded columns of one page (cached), from the block cache when the block is there."""
        bkey = self._key(ent)
        key = bkey + (int(page),)
        with self._lock:
            c = self._pages.get(key)
            if c is not None:
                self._pages.move_to_end(key)
                return c
            blk = self._cache.get(bkey)
        if blk is not None:
            return blk
        c = decode_block(self._read_pages(ent, page, page + 1), pages=(page, page + 1), check=False)
        with self._lock:
            self._pages[key] = c
            while len(self._pages) > self.cache_pages:
                self._pages.popitem(last=False)
        return c

    def _row_event(self, ent, row: int):
        """The event at ``row`` of a block, reading one page."""
        c = self._page_cols(ent, int(row) // PAGE_ROWS)
        return c, int(row) - int(c["row0"])

    # ------------------------------------------------------------------ reads
    def _decoded(self, ent) -> dict:
        key = self._key(ent)
        with self._lock:
            c = self._cache.get(key)
            if c is not None:
                self._cache.move_to_end(key)
                return c
        c = decode_block(self.seg.read_block(ent))
        with self._lock:
            self._cache[key] = c
            while len(self._cache) > self.cache_blocks:
                self._cache.popitem(last=False)
        return c

    def add_columnar(self, payload, wait: bool = True) -> int:
        """Event management's batch ingest (``add_columnar_batch``): a durable batch (GPU-encoded
        block) or a row batch (``persistence/columnar.py`` format, encoded here).  Returns the rows
        added (0 for a replay the store already holds) once they are on disk (``wait``)."""
        n, tok = self.add_batch(payload)
        if tok < 0:
            return 0
        if wait and not self.wait(tok):
            raise TimeoutError("event block not durable in time")
        return n

    def add_batch(self, payload) -> tuple[int, int]:
        """:meth:`add_columnar` without the wait: (rows, store token; -1 = a replay already held).
        The rows are durable once :meth:`durable` reaches the token."""
        if is_durable_batch(payload):
            d, blk = decode_durable_batch(payload)
            if len(blk) < 64:
                raise ValueError("durable batch without a block")
            n = int(blk[:64].view(HDR)[0]["n_rows"])
            # bytes crossed a process boundary (RPC / Kafka): check every page; an in-process view
            # of the engine's buffer was sealed here a moment ago
            if isinstance(payload, (bytes, bytearray, memoryview)) and verify(blk):
                raise ValueError("corrupt event block in a durable batch")
            owner = payload
            src = d.get("src") or None
            if src is not None and not int(blk[:64].view(HDR)[0]["flags"]) & FLAG_COMMIT:
                blk = blk.copy()                # the sender did not flag it: flag a copy
                set_commit_flag(blk)
                owner = blk
            tok = self.add_block(blk.ctypes.data, len(blk), owner=owner, boot=d["boot"], asg=d.get("asg"),
                                 names=d.get("names"), rules=d.get("rules"), src=src, ctx=d.get("ctx"))
        else:
            from .columnar import decode_batch
            d = decode_batch(payload)
            rows = d["rows"]
            n = len(rows)
            blk = encode_block(rows, index=True)       # zone maps; rows carry no strings / context ids
            seal(blk, int(d["first_seq"]), int(d["now"]), boot_id(d["boot"]), int(d["rank"]), int(d["world"]))
            src = d.get("src") or None
            if src is not None:
                set_commit_flag(blk)
            tok = self.add_block(blk.ctypes.data, len(blk), owner=blk, boot=d["boot"], asg=d.get("asg"),
                                 names=d.get("names"), rules=d.get("rules"), src=src)
        return (n, tok) if tok >= 0 else (0, -1)

    @property
    def rows(self) -> int:
        """Rows on disk (retention included)."""
        return int(self.seg.index()["n_rows"].sum())

    def count(self) -> int:
        return self.rows + self._objects.count()

    @property
    def api_boot(self) -> int:
        """The boot API-added events are stored under (see :meth:`add_events`)."""
        return self._api_boot

    @property
    def engine_rows(self) -> int:
        """Rows on disk that engines wrote (API-added events' blocks excluded)."""
        ents = self.seg.index()
        return int(ents["n_rows"][ents["boot"].astype(np.int64) != self._api_boot].sum())

    @staticmethod
    def _eids(h, idx) -> np.ndarray:
        return (int(h["first_seq"]) + np.asarray(idx, np.int64)) * int(h["world"]) + int(h["rank"])

    def get_event_by_id(self, id: str):
        boot, sep, num = id.rpartition("-")
        try:
            b = int(boot, 16)
        except ValueError:
            b = None
        ev = self._objects.get_event_by_id(id)     # the API tail first: it leaves only once a block holds it
        if ev is not None or not (sep and num.isdigit()) or b is None:
            return ev
        eid = int(num)
        ents = self.seg.index()
        if len(ents) and eid < (1 << 62):
            # event id = (first_seq + row) * world + rank: the block holding it, over all blocks at once
            w = np.maximum(ents["world"].astype(np.int64), 1)
            r = ents["rank"].astype(np.int64)
            row = (eid - r) // w - ents["first_seq"].astype(np.int64)
            hit = np.nonzero((ents["boot"].astype(np.int64) == b) & ((eid - r) % w == 0) & (row >= 0)
                             & (row < ents["n_rows"].astype(np.int64)))[0]
            if len(hit):
                e = ents[int(hit[0])]
                c, i = self._row_event(e, int(row[int(hit[0])]))
                return self._materialize(c, i)
        return None

    def list_command_responses_for_invocation(self, invocation_id, criteria=None):
        """Responses to an invocation, newest first: the tail's, and the blocks' response rows of the
        invocation's assignment (the assignment index) whose originating event is the invocation."""
        c = criteria or DateRangeSearchCriteria(page_size=100)
        tail = self._objects.list_command_responses_for_invocation(invocation_id, DateRangeSearchCriteria(
            page_size=0)).results
        inv = self.get_event_by_id(invocation_id)
        got = {e.id: e for e in tail}
        if inv is not None and inv.device_assignment_id:
            for e in self.list_events(DeviceEventType.CommandResponse, DeviceEventIndex.Assignment,
                                      [inv.device_assignment_id], DateRangeSearchCriteria(page_size=0)).results:
                if getattr(e, "originating_event_id", None) == invocation_id:
                    got.setdefault(e.id, e)
        out = sorted(got.values(), key=lambda ev: -(ev.event_date or 0))
        return SearchResults(len(out), c.slice(out))

    # ------------------------------------------------------------------ native point reads
    def _file_fds(self, files: np.ndarray, missing_ok: bool = False):
        """(fd per entry of ``files`` -- segment file ids -- opened read-only, the fds to close).
        ``missing_ok``: a file retention deleted after the caller took its block table gets fd -1
        (the caller drops those tasks, unless the store still holds the page in memory); otherwise
        KeyError."""
        uf, inv = np.unique(np.asarray(files, np.int64), return_inverse=True)
        opened, fds = [], []
        try:
            for f in uf.tolist():
                path = self.seg.file_path(int(f))
                fd = -1
                if path is not None:
                    try:
                        fd = os.open(path, os.O_RDONLY)
                    except FileNotFoundError:
                        fd = -1
                if fd < 0:
                    if not missing_ok:
                        raise KeyError("segment file deleted by retention")
                else:
                    opened.append(fd)
                fds.append(fd)
        except BaseException:
            for x in opened:
                os.close(x)
            raise
        return np.asarray(fds, np.int32)[inv.reshape(-1)], opened

    @property
    def _map_reserve(self) -> int:
        # a file ends with the first block past its rotation size: reserve one large block beyond it
        return self.rotate_bytes + (256 << 20)

    def _map_file(self, fid: int, end: int):
        """A read-only map (:class:`_FileMap`) of segment file ``fid`` covering at least its first
        ``end`` bytes, or None when the file is gone.  The map reserves the file's whole rotation
        size, so the file being appended to needs no new map as it grows: only pages of blocks the
        store has indexed (written) are ever read through it.  Maps are shared by the readers; a
        caller keeps the object it got for as long as it reads through the address (a dropped map is
        unmapped once no reader holds it).  Files are only appended to, and only cut back to their
        written bytes, so a map never loses a page it is read at."""
        import threading
        lock = self.__dict__.setdefault("_map_lock", threading.Lock())
        maps = self.__dict__.setdefault("_maps", {})
        path = self.seg.file_path(int(fid))
        if path is None:                  # retention deleted it: its rows are gone for this reader too
            with lock:
                maps.pop(fid, None)
            return None
        with lock:
            e = maps.get(fid)
            if e is not None and e.length >= end:
                return e
        try:
            fd = os.open(path, os.O_RDONLY)
        except FileNotFoundError:
            return None
        try:
            size = os.fstat(fd).st_size
            if size < end:
                return None
            e = _FileMap(fd, max(size, end, self._map_reserve))
        finally:
            os.close(fd)
        if not e.addr:
            return None
        with lock:
            maps[fid] = e
            if len(maps) > 1 and fid == max(maps):
                # a new file: forget the maps of files retention deleted
                for f in [f for f in maps if self.seg.file_path(int(f)) is None]:
                    del maps[f]
        return e

    def _mapped_pages(self, files, pos, nb, mem):
        """``mem`` with the address of every task's page in a map of its segment file where it had
        none (0 where the file is gone), and the maps to hold while reading."""
        mem = np.zeros(len(files), np.uint64) if mem is None else np.array(mem, np.uint64)
        need = np.nonzero(mem == 0)[0]
        held = []
        if not len(need):
            return mem, held
        f = np.asarray(files, np.int64)[need]
        p = np.asarray(pos, np.int64)[need]
        end = p + np.asarray(nb, np.int64)[need]
        uf, inv = np.unique(f, return_inverse=True)
        base = np.zeros(len(uf), np.uint64)
        for j, fid in enumerate(uf.tolist()):
            e = self._map_file(fid, int(end[inv == j].max()))
            if e is not None:
                held.append(e)
                base[j] = e.addr
        b = base[inv.reshape(-1)]
        mem[need] = np.where(b != 0, b + p.astype(np.uint64), np.uint64(0))
        return mem, held

    @staticmethod
    def _readable(fd: np.ndarray, mem) -> np.ndarray:
        """Tasks whose page can still be read: from its file, or from the store's memory copy."""
        ok = fd >= 0
        if mem is not None:
            ok |= np.asarray(mem, np.uint64) != 0
        return ok

    def _page_geometry(self, t, bis: np.ndarray, pages: np.ndarray, scan: bool = False):
        """(file id, file offset, bytes, rows) of pages ``pages`` of blocks ``bis`` (positions in t)."""
        n = len(bis)
        ents = t["ents"]
        bis, pages = np.ascontiguousarray(bis, np.int64), np.ascontiguousarray(pages, np.int64)
        off, nb = np.empty(n, np.uint32), np.empty(n, np.uint32)
        miss = int(native().swseg_ix_page_geom(t["addr"], t["n"], _p(bis), _p(pages), n, _p(off), _p(nb)))
        if miss:                                      # blocks without a trailer: their page headers
            for bi in np.unique(bis[nb == 0]).tolist():
                m = bis == bi
                pg = self._pages_of(ents[bi], t["tr"][bi])
                off[m] = pg["off"][pages[m]]
                nb[m] = pg["bytes"][pages[m]]
        pos = ents["offset"][bis].astype(np.int64) + off.astype(np.int64)
        n_rows = ents["n_rows"][bis].astype(np.int64)
        rows = np.minimum(PAGE_ROWS, n_rows - pages * PAGE_ROWS).astype(np.uint32)
        # scans read the pages' prefixes from the scan images the store holds (0: from the file)
        mem = np.zeros(n, np.uint64)
        if scan and "baddr" in t and n:
            ba = np.ascontiguousarray(t["baddr"], np.uint64)
            native().swseg_image_addrs(_p(ba), _p(bis), _p(pages), n, _p(mem))
        return ents["file"][bis].astype(np.int64), pos, nb, rows, mem

    def _fetch(self, t, bis, rows) -> dict:
        """Decoded columns (+ strings, + per-row block fields for :func:`materialize_row`) of rows
        (block position, row) of one boot table, in request order: each page read and checked once
        (native ``swseg_fetch_rows``, multi-threaded), only the requested rows kept."""
        bis, rows = np.asarray(bis, np.int64), np.asarray(rows, np.int64)
        n = len(bis)
        pages = rows // PAGE_ROWS
        order = np.lexsort((pages, bis))
        sb, sp = bis[order], pages[order]
        files, pos, nb, prows, mem = self._page_geometry(t, sb, sp)
        rip = (rows[order] - sp * PAGE_ROWS).astype(np.int32)
        cols = {"etype": np.empty(n, np.uint8), "level": np.empty(n, np.uint8), "date": np.empty(n, np.int64),
                "asg": np.empty(n, np.int32), "name": np.empty(n, np.uint16), "v0": np.empty(n, np.float64),
                "v1": np.empty(n, np.float64), "v2": np.empty(n, np.float64), "flags": np.empty(n, np.uint8)}
        offs = np.zeros(3 * n + 1, np.int64)
        fd, opened = self._file_fds(files)
        try:
            cap = 2048 * max(1, n)
            while True:
                heap = np.empty(cap, np.uint8)
                k = int(native().swseg_fetch_rows(
                    _p(fd), _p(pos), _p(nb), _p(prows), _p(rip), n, min(self.scan_threads, 8),
                    *[_p(cols[c]) for c in ("etype", "level", "date", "asg", "name", "v0", "v1", "v2", "flags")],
                    _p(heap), cap, _p(offs), _p(mem)))
                if k >= 0:
                    break
                if k <= -(1 << 40):
                    cap = -k - (1 << 40) + 64
                    continue
                raise ValueError(f"corrupt or unreadable event page (request {-k - 1})")
        finally:
            for x in opened:
                os.close(x)
        inv = np.empty(n, np.int64)
        inv[order] = np.arange(n)
        # back to request order (strings: offsets of request i are those of sorted position inv[i])
        out = {c: v[inv] for c, v in cols.items()}
        lens = np.diff(offs).reshape(n, 3)[inv]         # (alt id, message, metadata) bytes per request
        so = np.zeros(3 * n + 1, np.int64)
        so[1:] = np.cumsum(lens.reshape(-1))
        per_row = lens.sum(axis=1)
        # byte p of request i's strings comes from its sorted position's strings at the same distance
        src = np.repeat(offs[3 * inv] - so[0:3 * n:3], per_row) + np.arange(int(per_row.sum()))
        out["str_heap"], out["str_off"] = heap[src], so
        e = t["ents"][bis]
        out.update(rows=rows, boot=e["boot"].astype(np.int64), first_seq=e["first_seq"].astype(np.int64),
                   world=e["world"].astype(np.int64), rank=e["rank"].astype(np.int64),
                   recv_ms=e["recv_ms"].astype(np.int64))
        return out

    def _alt_page_rows(self, t, bis, pages, hashes) -> tuple[np.ndarray, np.ndarray]:
        """(candidate index, row in block) of the rows whose alternate-id hash matches, over candidate
        pages (block position, page, hash) of one boot table (native ``swseg_alt_page_rows``)."""
        bis, pages = np.asarray(bis, np.int64), np.asarray(pages, np.int64)
        n = len(bis)
        if not n:
            return np.zeros(0, np.int64), np.zeros(0, np.int64)
        files, pos, nb, prows, mem = self._page_geometry(t, bis, pages)
        hv = np.asarray(hashes, np.uint64)
        fd, opened = self._file_fds(files, missing_ok=True)
        keep = self._readable(fd, mem)
        if not keep.all():             # retention deleted a file meanwhile: its ids are no longer stored
            sel = np.nonzero(keep)[0]
            pages = pages[sel]
            fd, pos, nb, prows, hv = fd[sel], pos[sel], nb[sel], prows[sel], hv[sel]
            mem = mem[sel] if mem is not None else None
            n = len(sel)
            if not n:
                for x in opened:
                    os.close(x)
                return np.zeros(0, np.int64), np.zeros(0, np.int64)
        else:
            sel = None
        try:
            cap = max(16, n)
            while True:
                ot, orow = np.empty(cap, np.int64), np.empty(cap, np.int32)
                k = int(native().swseg_alt_page_rows(_p(fd), _p(pos), _p(nb), _p(prows), _p(hv), n,
                                                     min(self.scan_threads, 8), _p(ot), _p(orow), cap, _p(mem)))
                if k < 0:
                    raise ValueError(f"corrupt or unreadable event page (candidate {-k - 1})")
                if k <= cap:
                    break
                cap = k
        finally:
            for x in opened:
                os.close(x)
        ci = ot[:k] if sel is None else sel[ot[:k]]
        return ci, pages[ot[:k]] * PAGE_ROWS + orow[:k].astype(np.int64)

    # ------------------------------------------------------------------ listings
    def _pages_of(self, ent, tr):
        """SwIxPage rows of a block (from its trailer, or its page headers when it has none)."""
        if tr is not None:
            th, view = tr[2], tr[3]
            o = int(th["off_pages"])
            return view[o:o + 32 * int(th["n_pages"])].view(IX_PAGE)
        blk = self.seg.read_block(ent)
        ps = page_summary(blk)
        pt = blk[64:64 + 4 * (len(ps) + 1)].view(np.uint32)
        out = np.zeros(len(ps), IX_PAGE)
        out["asg_min"], out["asg_max"], out["date_min"], out["date_max"] = ps[:, 2], ps[:, 3], ps[:, 4], ps[:, 5]
        out["off"], out["bytes"] = pt[:-1], np.diff(pt)
        return out

    def _scan_pages(self, t, bis, pages, et: int, d_lo: int, d_hi: int, asg: int = -1, ctx_tab=None,
                    ctx_id: int = 0, asg_list=None, task_lo=None, task_hi=None, sorted_=None):
        """Rows of pages ``pages`` of blocks ``bis`` (positions in boot table t) passing (type, date
        range, assignment | context id | one of the sorted ``asg_list[task_lo[i]:task_hi[i]]`` per
        page), reading each page's leading columns only (native ``swseg_scan_pages``,
        multi-threaded) -> (block position, row in block, date) arrays."""
        bis, pages = np.asarray(bis, np.int64), np.asarray(pages, np.int64)
        if not len(bis):
            return np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(0, np.int64)
        files, pos, nb, _, mem = self._page_geometry(t, bis, pages, scan=True)
        # pages read in place through maps of their files (no read call and copy per page); a page
        # whose file is gone is read from the store's scan image, or dropped
        mem, held = self._mapped_pages(files, pos, nb, mem)
        fd, opened = self._file_fds(files[mem == 0], missing_ok=True)
        fd_all = np.full(len(files), -1, np.int32)
        fd_all[mem == 0] = fd
        fd = fd_all
        keep = self._readable(fd, mem)
        if not keep.all():             # retention deleted a file meanwhile: its rows are gone
            sel = np.nonzero(keep)[0]
            bis, pages, fd, pos, nb = bis[sel], pages[sel], fd[sel], pos[sel], nb[sel]
            mem = mem[sel] if mem is not None else None
            if asg_list is not None:
                task_lo, task_hi = np.ascontiguousarray(task_lo[sel]), np.ascontiguousarray(task_hi[sel])
            if sorted_ is not None:
                sorted_ = np.ascontiguousarray(sorted_[sel])
            if not len(sel):
                for x in opened:
                    os.close(x)
                return np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(0, np.int64)
        poff = np.zeros(len(bis), np.uint32)
        pix = pages.astype(np.int32)
        ct = np.ascontiguousarray(ctx_tab, np.int32) if ctx_tab is not None else np.zeros(1, np.int32)
        try:
            cap = 4096
            while True:
                ot, orow, od = np.empty(cap, np.int64), np.empty(cap, np.int32), np.empty(cap, np.int64)
                k = int(native().swseg_scan_pages(_p(fd), _p(pos), _p(poff), _p(nb), _p(pix), len(bis), int(et),
                                                  int(asg), _p(ct), len(ct) if ctx_tab is not None else 0, int(ctx_id),
                                                  int(d_lo), int(d_hi), self.scan_threads, _p(ot), _p(orow), _p(od), cap,
                                                  _p(mem), _p(asg_list) if asg_list is not None else None,
                                                  _p(task_lo) if asg_list is not None else None,
                                                  _p(task_hi) if asg_list is not None else None,
                                                  _p(sorted_) if sorted_ is not None else None))
                if k < 0:
                    raise ValueError(f"event page unreadable (task {-k - 1})")
                if k <= cap:
                    return bis[ot[:k]], orow[:k].astype(np.int64), od[:k]
                cap = k
        finally:
            for f in opened:
                os.close(f)

    def _rows_for(self, t, blocks, et, d_lo, d_hi, asg=-1, ctx_tab=None, ctx_id=0):
        """(block position, row, date) of every matching row of the listed blocks (the pages whose
        zone maps admit the date range, and ``asg`` when given)."""
        bl, pl = [], []
        for bi in blocks:
            pg = self._pages_of(t["ents"][bi], t["tr"][bi])
            m = (pg["date_max"] >= d_lo) & (pg["date_min"] <= d_hi)
            if asg >= 0:
                m &= (pg["asg_min"] <= asg) & (pg["asg_max"] >= asg)
            p = np.nonzero(m)[0]
            bl.append(np.full(len(p), bi, np.int64))
            pl.append(p)
        if not bl:
            return np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(0, np.int64)
        return self._scan_pages(t, np.concatenate(bl), np.concatenate(pl), et, d_lo, d_hi, asg, ctx_tab, ctx_id)

    def _asg_pages(self, t, asg: int, d_lo: int, d_hi: int) -> tuple[np.ndarray, np.ndarray]:
        """(block positions, pages) whose assignment / date zone maps admit the assignment."""
        cap = max(1024, 4 * t["n"])
        bo, po = np.empty(cap, np.int64), np.empty(cap, np.int64)
        k = int(native().swseg_ix_asg_pages(t["addr"], t["n"], int(asg), int(d_lo), int(d_hi), _p(bo), _p(po), cap))
        if k > cap:
            bo, po = np.empty(k, np.int64), np.empty(k, np.int64)
            k = int(native().swseg_ix_asg_pages(t["addr"], t["n"], int(asg), int(d_lo), int(d_hi), _p(bo), _p(po), k))
        return bo[:k], po[:k]

    def _list_assignments(self, t, asg_idx, et, d_lo, d_hi) -> tuple[int, list]:
        """Rows of the assignments over one boot's blocks: the blocks are clustered by assignment, so
        the page zone maps name one or two pages per block, read as their leading columns."""
        parts = []
        legacy = [bi for bi, tr in enumerate(t["tr"]) if tr is None]
        for a in asg_idx:
            bo, po = self._asg_pages(t, a, d_lo, d_hi)
            b, rows, dates = self._scan_pages(t, bo, po, et, d_lo, d_hi, asg=int(a))
            if len(b):
                parts.append((b, rows, dates))
            if legacy:
                parts.append(self._rows_for(t, legacy, et, d_lo, d_hi, asg=int(a)))
        return self._collect(t, parts)

    @staticmethod
    def _collect(t, parts) -> tuple[int, list]:
        if not parts:
            return 0, []
        bi = np.concatenate([p[0] for p in parts])
        rows = np.concatenate([p[1] for p in parts])
        dates = np.concatenate([p[2] for p in parts])
        eids = (t["first"][bi] + rows) * t["world"][bi] + t["rank"][bi]
        return len(rows), [(dates, eids, bi, rows, t)]

    def _ctx_table(self, boot: int, pos: int) -> np.ndarray | None:
        """Context id (dimension pos - 2) by assignment index for one boot, from the dictionaries
        (kept current by :meth:`_apply_dict`); None when the boot's context ids are unknown."""
        if not self._ctx.get(boot, {}).get(pos - 2):
            return None
        arr = self._ctx_arr.get(boot)
        if arr is None:
            return None
        return arr[pos - 2, :self._asg_n.get(boot, 0)]

    def _ctx_via_assignments(self, t, ctx_tab, cid: int, mask, et, d_lo, d_hi):
        """(block position, row, date) of context id ``cid`` in the masked blocks, found through its
        assignments: one native pass maps them to the pages their zone maps admit
        (``swseg_ix_asgs_pages``), one native scan of those pages' leading columns keeps the rows of
        the id (the reference's Mongo (asset | customer, type, date) index at any cardinality,
        MongoDeviceEventManagement.java:132-140)."""
        t0 = time.perf_counter()
        asgs = np.ascontiguousarray(np.nonzero(ctx_tab == cid)[0], np.int32)
        if not len(asgs):
            return np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(0, np.int64)
        m = np.ascontiguousarray(mask, np.uint8)
        cap = max(1024, 4 * len(asgs))
        while True:
            bo, po = np.empty(cap, np.int64), np.empty(cap, np.int64)
            lo, hi = np.empty(cap, np.int64), np.empty(cap, np.int64)
            srt = np.empty(cap, np.uint8)
            k = int(native().swseg_ix_asgs_pages(t["addr"], t["n"], _p(asgs), len(asgs), _p(m), int(d_lo), int(d_hi),
                                                 _p(bo), _p(po), cap, _p(lo), _p(hi), _p(srt)))
            if k <= cap:
                break
            cap = k
        t1 = time.perf_counter()
        # each page is scanned for the id's assignments its zone map admits (no context table lookup);
        # a sorted page (its block's trailer says SIX_F_CLUSTERED) by binary search
        r = self._scan_pages(t, bo[:k], po[:k], et, d_lo, d_hi, asg_list=asgs, task_lo=np.ascontiguousarray(lo[:k]),
                             task_hi=np.ascontiguousarray(hi[:k]), sorted_=np.ascontiguousarray(srt[:k]))
        ph = getattr(self._tl, "phases", None)
        if ph is not None:                            # sub-phases of "index" (read-load reports)
            t2 = time.perf_counter()
            ph["ix_pages"] = ph.get("ix_pages", 0.0) + t1 - t0
            ph["ix_scan"] = ph.get("ix_scan", 0.0) + t2 - t1
            ph["ix_scan_pages_n"] = ph.get("ix_scan_pages_n", 0) + k              # counts, not seconds
            ph["ix_scan_sorted_n"] = ph.get("ix_scan_sorted_n", 0) + int(srt[:k].sum())
        return r

    def _list_context(self, t, boot, pos, want, et, d_lo, d_hi, need) -> tuple[int, list]:
        """Rows of customer / area / asset ids over one boot's blocks, from the trailers' key tables:
        exact totals from the per-key counts (a block straddling a date bound is scanned for its
        count), the newest rows from the per-key heads merged across blocks; a block whose heads the
        merge runs past is scanned."""
        d = pos - 2
        ids = self._ctx.get(boot, {}).get(d, {})
        ctx_tab = self._ctx_table(boot, pos)
        bounded = d_lo > -(1 << 62) or d_hi < (1 << 62)
        if ctx_tab is None:                           # no context ids for this boot: via assignments
            asg_idx = [i for i, ctx in self._asg.get(boot, {}).items() if len(ctx) > pos and ctx[pos] in want]
            return self._list_assignments(t, asg_idx, et, d_lo, d_hi)
        lib = native()
        n = t["n"]
        total, parts, heads = 0, [], []
        maybe = []                                    # (block, last head date, last head eid, cid)
        scan = {}                                     # block -> ctx ids to scan it for
        for tok in want:
            cid = ids.get(tok)
            if cid is None:
                continue
            out = np.zeros(7 * n, np.int64)
            cap = 16 * n + 16
            while True:
                hb, hr, hd = np.empty(cap, np.int64), np.empty(cap, np.int64), np.empty(cap, np.int64)
                k = int(lib.swseg_ix_ctx_heads(t["addr"], n, d, (int(cid) << 3) | int(et), _p(out), _p(hb), _p(hr),
                                               _p(hd), cap))
                if k <= cap:
                    break
                cap = k
            o = out.reshape(n, 7)
            st, cnt, dmin, dmax, h0, nh = o[:, 0], o[:, 1], o[:, 2], o[:, 3], o[:, 4], o[:, 5]
            outside = (dmax < d_lo) | (dmin > d_hi)
            straddle = bounded & ~outside & ~((d_lo <= dmin) & (dmax <= d_hi))
            # blocks that do not index this dimension (its context ids passed SIX_CTX_MAX: an asset
            # per device, 10K customers): through the id's assignments and their pages' zone maps
            notix = (st < 0) & np.fromiter((tr is not None for tr in t["tr"]), bool, n)
            if notix.any():
                b, r, dt = self._ctx_via_assignments(t, ctx_tab, int(cid), notix, et, d_lo, d_hi)
                total += len(r)
                heads.append((b, r, dt))
            to_scan = ((st < 0) & ~notix) | ((st > 0) & straddle)   # no trailer / straddles a bound
            for bi in np.nonzero(to_scan)[0].tolist():
                scan.setdefault(bi, set()).add(int(cid))
            use = (st > 0) & ~to_scan & ~outside
            total += int(cnt[use].sum())
            keep = use[hb[:k]]
            heads.append((hb[:k][keep], hr[:k][keep], hd[:k][keep]))
            for bi in np.nonzero(use & (cnt > nh))[0].tolist():
                j = int(h0[bi] + nh[bi] - 1)
                maybe.append((bi, int(hd[j]), int(hr[j]), int(cid)))
        # blocks to scan in full (exact rows): not indexed, straddling a date bound, or heads exhausted
        def scan_blocks(blks):
            got = []
            for bi, cids in blks.items():
                for cid in cids:
                    b, r, dt = self._rows_for(t, [bi], et, d_lo, d_hi, ctx_tab=ctx_tab, ctx_id=cid)
                    got.append((b, r, dt))
            return got
        scanned = scan_blocks(scan)
        total += sum(len(x[1]) for x in scanned)
        cand = heads + scanned
        if maybe and need > 0:
            # the cutoff of the merged heads: a block whose last head is above it may hold more
            bi_ = np.concatenate([c[0] for c in cand]) if cand else np.zeros(0, np.int64)
            rows_ = np.concatenate([c[1] for c in cand]) if cand else np.zeros(0, np.int64)
            dates_ = np.concatenate([c[2] for c in cand]) if cand else np.zeros(0, np.int64)
            eids_ = ((t["first"][bi_] + rows_) * t["world"][bi_] + t["rank"][bi_]) if len(bi_) else \
                np.zeros(0, np.int64)
            if len(dates_) >= need:
                order = np.lexsort((-eids_, -dates_))
                cut = order[need - 1]
                cut_d, cut_e = int(dates_[cut]), int(eids_[cut])
            else:
                cut_d, cut_e = None, None
            more: dict = {}
            all_cids = {int(ids[tok]) for tok in want if tok in ids}
            for bi, ld, lr, cid in maybe:
                le = (int(t["first"][bi]) + lr) * int(t["world"][bi]) + int(t["rank"][bi])
                if cut_d is None or (ld, le) > (cut_d, cut_e):
                    more[bi] = all_cids          # the block is rescanned whole: every wanted id
            if more:
                extra = scan_blocks(more)
                if cand:
                    b = np.concatenate([c[0] for c in cand])
                    keep = ~np.isin(b, np.fromiter(more, np.int64))
                    cand = [(b[keep], np.concatenate([c[1] for c in cand])[keep],
                             np.concatenate([c[2] for c in cand])[keep])]
                cand += extra
        return total, self._collect(t, cand)[1]

    @_leased
    def list_events(self, event_type, index, entity_ids, criteria: DateRangeSearchCriteria | None = None):
        """Events of one type for entities of an index, newest first, with the exact total.
        Assignment: page zone maps of the assignment-clustered blocks, then those pages' leading
        columns.  Customer / area / asset: the trailers' per-key counts and heads (see
        :meth:`_list_context`).  API-added events join from their own store."""
        c = criteria or DateRangeSearchCriteria(page_size=100)
        et = _ETYPE.get(DeviceEventType(event_type))
        clock = time.perf_counter
        ph = self._tl.phases = {}                     # where the call's time went (read-load reports)
        t0 = clock()
        objs = self._objects.list_events(event_type, index, entity_ids, DateRangeSearchCriteria(
            page_size=0, start_date=c.start_date, end_date=c.end_date)).results
        if et is None:
            return SearchResults(len(objs), c.slice(objs))
        pos = _CTX[DeviceEventIndex(index)]
        want = set(entity_ids)
        paged = c.page_size > 0
        need = max(1, c.page_number) * c.page_size if paged else 1 << 62
        d_lo = c.start_date if c.start_date is not None else -(1 << 62)
        d_hi = c.end_date if c.end_date is not None else (1 << 62)
        total = len(objs)
        found = []                                    # (dates, eids, block positions, rows, table)
        tabs = self._boot_tables()
        covered = self._api_covered(tabs)             # tail events a block now holds: counted there
        if covered and objs:
            objs = [e for e in objs if self._api_seq(e) < 0 or self._api_seq(e) >= covered]
            total = len(objs)
        t1 = clock()
        ph["tables"] = t1 - t0
        for b, t in tabs.items():
            if pos == 0:
                with self._lock:
                    tok = self._asg_tok.get(b, {})
                    asg_idx = sorted({i for w in want for i in tok.get(w, ())})
                n, parts = self._list_assignments(t, asg_idx, et, d_lo, d_hi)
            else:
                n, parts = self._list_context(t, b, pos, want, et, d_lo, d_hi, need)
            total += n
            found.extend(parts)
        t2 = clock()
        ph["index"] = t2 - t1
        if not found:
            return SearchResults(total, c.slice(objs))
        dates = np.concatenate([x[0] for x in found])
        eids = np.concatenate([x[1] for x in found])
        which = np.concatenate([np.full(len(x[0]), k, np.int32) for k, x in enumerate(found)])
        pos_ = np.concatenate([x[2] for x in found])
        rows = np.concatenate([x[3] for x in found])
        order = np.lexsort((-eids, -dates))

        def mat(sel):
            """The events of the selected candidates, read together (one native fetch per boot)."""
            evs = [None] * len(sel)
            tabs = [found[int(k)][4] for k in which[sel]]
            groups: dict = {}
            for j, t in enumerate(tabs):
                groups.setdefault(id(t), (t, []))[1].append(j)
            t3 = clock()
            ph["order"] = t3 - t2
            for t, js in groups.values():
                cols = self._fetch(t, pos_[sel[js]], rows[sel[js]])
                t4 = clock()
                ph["fetch"] = ph.get("fetch", 0.0) + t4 - t3
                for m, j in enumerate(js):
                    evs[j] = self._materialize(cols, m)
                t3 = clock()
                ph["materialize"] = ph.get("materialize", 0.0) + t3 - t4
            return evs
        if objs:
            if paged:
                order = order[:need + len(objs)]
            merged = mat(order) + objs
            merged.sort(key=lambda ev: -(ev.event_date or 0))
            return SearchResults(total, c.slice(merged))
        if paged:
            start = (max(1, c.page_number) - 1) * c.page_size
            order = order[start:start + c.page_size]
        return SearchResults(total, mat(order))

    def _materialize(self, cols: dict, i: int):
        b = int(cols["boot"][i]) if "rows" in cols else cols["header"]["boot"]
        return materialize_row(cols, i, self._asg.get(b, {}), self._names.get(b, {}), self._rules)

    def dictionary(self, boot, asg_ids=(), name_ids=()) -> dict:
        """Dictionary entries of an engine incarnation (assignment index -> context, name id -> name)
        and the rule messages: what an enriched-batch consumer that started after the batch carrying
        them needs to materialize rows."""
        b = boot_id(boot)
        with self._lock:
            a, n = self._asg.get(b, {}), self._names.get(b, {})
            return {"asg": {int(i): a[int(i)] for i in asg_ids if int(i) in a},
                    "names": {int(i): n[int(i)] for i in name_ids if int(i) in n}, "rules": dict(self._rules)}


def materialize_row(cols: dict, i: int, asg: dict, names: dict, rules: dict):
    """Decoded block row ``i`` -> the reference event: ids and assignment context (``asg``: index ->
    [assignment, device, customer, area, asset, ...]), alternate id, metadata, and per type the name /
    value, coordinates (elevation when sent), alert source / level / type / message, or the
    engine's presence state change.  ``names``: name id -> name; ``rules``: rule alert type -> message."""
    if "rows" in cols:           # rows fetched across blocks (DurableEventStore._fetch): per-row block fields
        h = {"boot": int(cols["boot"][i]), "first_seq": int(cols["first_seq"][i]), "world": int(cols["world"][i]),
             "rank": int(cols["rank"][i]), "recv_ms": int(cols["recv_ms"][i])}
        row = int(cols["rows"][i])
    else:
        h = cols["header"]
        row = int(cols.get("row0", 0)) + i
    b = h["boot"]
    ctx = asg.get(int(cols["asg"][i])) or [None] * 5
    eid = (h["first_seq"] + row) * h["world"] + h["rank"]
    alt, msg, md = row_strings(cols, i)
    f = int(cols["flags"][i])
    base = dict(id=f"{b:x}-{eid}", device_assignment_id=ctx[0], device_id=ctx[1], customer_id=ctx[2],
                area_id=ctx[3], asset_id=ctx[4], event_date=int(cols["date"][i]), received_date=h["recv_ms"],
                alternate_id=alt, metadata=md)
    et = int(cols["etype"][i])
    nid = int(cols["name"][i])
    name = names.get(nid, "") if nid != NO_NAME else ""
    if f & SEGF_JSON:                 # an API-added invocation / response / state change (api_blocks.py)
        from .api_blocks import event_from_json_row
        return event_from_json_row(et, json.loads(_str(cols, i, 2) or b"{}"), base)
    if et == EV_MEASUREMENT:
        return DeviceMeasurement(name=name, value=float(cols["v0"][i]), **base)
    if et == EV_LOCATION:
        return DeviceLocation(latitude=float(cols["v0"][i]), longitude=float(cols["v1"][i]),
                              elevation=float(cols["v2"][i]) if f & SEGF_HAS_ELEV else None, **base)
    if et == EV_ALERT:
        gen = bool(f & SEGF_GEN)
        return DeviceAlert(source=AlertSource.System if gen or f & SEGF_SYS else AlertSource.Device,
                           level=_LEVELS[min(int(cols["level"][i]), 3)], type=name,
                           message=(rules.get(name) or "") if gen else msg, **base)
    # the engine's state changes are its presence scan (DevicePresenceManager.java:110-200)
    return DeviceStateChange(attribute="presence", type="presence", previous_state="PRESENT",
                             new_state="NOT_PRESENT", **base)
