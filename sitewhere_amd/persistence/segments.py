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

import ctypes
import json
import os
import threading
import time
import zlib
from collections import OrderedDict

import numpy as np

from .._native import native
from ..models.columnar import EV_ALERT, EV_LOCATION, EV_MEASUREMENT, EV_STATE_CHANGE, NO_NAME, OUT_REC
from ..models.domain import (AlertLevel, AlertSource, DateRangeSearchCriteria, DeviceAlert, DeviceEventIndex,
                             DeviceEventType, DeviceLocation, DeviceMeasurement, DeviceStateChange, SearchResults,
                             event_from_dict)
from .events import DeviceEventStore, MemoryEventStore

# SEG_FLAGS bits (csrc/include/swseg.h)
SEGF_HAS_US, SEGF_US, SEGF_HAS_ELEV, SEGF_HAS_ALT, SEGF_HAS_META, SEGF_GEN = 0x1, 0x2, 0x4, 0x8, 0x10, 0x20
SEG_ALIGN = 4096
PAGE_ROWS = 1024
PAGE_HDR = 400              # sizeof(SwSegPageHdr), csrc/include/swseg.h
FLAG_COMMIT = 1             # the block is followed by a commit record of input offsets (swseg.h)
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
IX_HDR = np.dtype([("magic", "<u4"), ("version", "<u2"), ("n_dims", "<u2"), ("n_rows", "<u4"), ("n_pages", "<u4"),
                   ("bytes", "<u8"), ("checksum", "<u8"), ("alt_bits", "<u4"), ("alt_pbits", "<u4"), ("n_alt", "<u4"),
                   ("off_pages", "<u4"), ("off_alt_dir", "<u4"), ("off_alt", "<u4"), ("off_keys", "<u4", 3),
                   ("n_keys", "<u4", 3), ("off_heads", "<u4", 3), ("n_heads", "<u4", 3), ("off_hdates", "<u4", 3),
                   ("pad", "<u4", 3)])
assert IX_HDR.itemsize == 128
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
    md = parse_metadata(_str(cols, i, 2), _META_FIELD.get(int(cols["etype"][i]), 0)) if f & SEGF_HAS_META else {}
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


def _durable_head(boot, asg: dict, names: dict, rules: dict | None, src=None) -> bytes:
    import msgpack
    import struct
    d = {"boot": boot_id(boot), "asg": {int(k): list(v) for k, v in (asg or {}).items()},
         "names": {int(k): v for k, v in (names or {}).items()}, "rules": rules or {}}
    if src:
        d["src"] = [[str(t), int(p), int(o)] for t, p, o in src]
    hdr = msgpack.packb(d, use_bin_type=True)
    head = DURABLE_MAGIC + struct.pack("<I", len(hdr)) + hdr
    return head + bytes(-len(head) % 64)


def encode_durable_batch(block: np.ndarray, boot, asg: dict | None = None, names: dict | None = None,
                         rules: dict | None = None, src=None) -> bytes:
    """``src``: ``[(topic, partition, next offset)]`` of the input the block completes (the block
    should then carry ``FLAG_COMMIT``, see :func:`set_commit_flag`)."""
    return _durable_head(boot, asg, names, rules, src) + memoryview(np.ascontiguousarray(block, np.uint8)).cast("B")


def frame_durable_batch(frame: tuple, nbytes: int, boot, asg: dict | None = None, names: dict | None = None,
                        rules: dict | None = None, src=None) -> np.ndarray | None:
    """Zero-copy :func:`encode_durable_batch` for a block at ``offset`` of ``buffer`` (``frame``)
    with free bytes in front of it; None when the header does not fit."""
    buf, off = frame
    head = _durable_head(boot, asg, names, rules, src)
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
        a = np.zeros(8, np.int64)
        self.lib.swss_stats(self.h, _p(a))
        return dict(zip(("bytes_written", "blocks_written", "syncs", "deleted_files", "deleted_bytes", "retained_bytes",
                         "files", "direct_io"), (int(x) for x in a)))

    def index(self) -> np.ndarray:
        cap = 1024
        while True:
            out = np.zeros(cap, INDEX_ENT)
            n = int(self.lib.swss_index(self.h, _p(out), cap))
            if n <= cap:
                return out[:n]
            cap = n + 1024

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
          DeviceEventType.Alert: EV_ALERT, DeviceEventType.StateChange: EV_STATE_CHANGE}
_LEVELS = [AlertLevel.Info, AlertLevel.Warning, AlertLevel.Error, AlertLevel.Critical]
_CTX = {DeviceEventIndex.Assignment: 0, DeviceEventIndex.Customer: 2, DeviceEventIndex.Area: 3,
        DeviceEventIndex.Asset: 4}


def boot_id(boot) -> int:
    """Numeric engine incarnation of a tenant's boot string (hex ms timestamp) or number."""
    return int(boot, 16) if isinstance(boot, str) else int(boot or 0)


class BlockIndex:
    """Indexes of one durable block (``swseg_index_block``), kept as memory-mapped ``.npy`` sidecars
    under ``<store>/index/<file>-<offset>.*``:

    * postings, one per row, sorted by (``pk`` = assignment index << 3 | event type, event date desc,
      row desc); ``pd`` = date - ``min_date`` (u32; ``wide`` when some date does not fit: such a
      block is answered by a scan), ``pr`` = row
    * alternate ids: ``ah`` = 64-bit hash of the full id (the engine's dedup hash, sorted), ``ar`` = row

    24 B per row; a lookup is a binary search per block, so a query over a billion stored events
    touches a few pages of these files per block instead of decoding the blocks."""

    PARTS = ("pk", "pd", "pr", "ah", "ar")
    __slots__ = PARTS + ("wide", "min_date")

    def __init__(self, pk, pd, pr, ah, ar, wide: bool, min_date: int):
        self.pk, self.pd, self.pr, self.ah, self.ar = pk, pd, pr, ah, ar
        self.wide, self.min_date = bool(wide), int(min_date)

    @property
    def nbytes(self) -> int:
        return sum(int(getattr(self, k).nbytes) for k in self.PARTS)

    @classmethod
    def build(cls, block: np.ndarray, min_date: int) -> "BlockIndex":
        n = int(header(block)["n_rows"])
        pk, pd, pr = np.empty(n, np.uint32), np.empty(n, np.uint32), np.empty(n, np.uint32)
        ah, ar = np.empty(n, np.uint64), np.empty(n, np.uint32)
        wide = np.zeros(1, np.int32)
        na = int(native().swseg_index_block(_p(block), int(min_date), _p(pk), _p(pd), _p(pr), _p(ah), _p(ar),
                                            _p(wide)))
        if na < 0:
            raise ValueError("event block index failed")
        return cls(pk, pd, pr, ah[:na], ar[:na], bool(wide[0]), min_date)

    def save(self, base: str):
        for k in self.PARTS:
            tmp = f"{base}.{k}.tmp.npy"
            np.save(tmp, np.ascontiguousarray(getattr(self, k)))
            os.replace(tmp, f"{base}.{k}.npy")
        with open(f"{base}.meta.tmp", "w") as f:             # written last: the index is complete
            json.dump({"wide": self.wide, "min_date": self.min_date}, f)
        os.replace(f"{base}.meta.tmp", f"{base}.meta")

    @classmethod
    def load(cls, base: str) -> "BlockIndex | None":
        try:
            with open(f"{base}.meta") as f:
                m = json.load(f)
            arrs = [np.load(f"{base}.{k}.npy", mmap_mode="r") for k in cls.PARTS]
        except (OSError, ValueError):
            return None
        return cls(*arrs, m["wide"], m["min_date"])

    @classmethod
    def remove(cls, base: str):
        for suffix in [f".{k}.npy" for k in cls.PARTS] + [".meta"]:
            try:
                os.remove(base + suffix)
            except OSError:
                pass


class DurableEventStore(DeviceEventStore):
    """Event store of engine tenants on durable segments (see module docstring).

    Ingest: :meth:`add_block` (an encoded, sealed block + the dictionary deltas its rows need).
    Events are identified by (boot, rank, store sequence): a block whose rows the store already
    holds for its (boot, rank) is skipped (a shard replaying after a restore).  Assignment and name
    indices are engine-local, so the dictionaries are kept per boot; their deltas are fsync'd to
    ``dict-<rank>.log`` before the block is queued, so a durable block never refers to an unknown
    entry."""

    def __init__(self, directory: str, rank: int = 0, rotate_bytes: int = 1 << 30, retention_bytes: int = 0,
                 direct: bool = True, cache_blocks: int = 8, index: bool = True, index_threads: int | None = None):
        self.dir = directory
        os.makedirs(directory, exist_ok=True)
        self.seg = SegmentStore(directory, rank, rotate_bytes, retention_bytes, direct)
        # events added through the API (REST / RPC adds, command invocations and responses, rule and
        # presence alerts): a checksummed JSON-lines log, fdatasync'd before the add returns, replayed
        # into the in-memory indexes on open
        self._objects = MemoryEventStore()
        self._api_path = os.path.join(directory, f"api-{rank}.log")
        self._load_api_log()
        self._api_f = open(self._api_path, "ab")
        self._asg: dict[int, dict[int, list]] = {}       # boot -> assignment index -> [asg, dev, cust, area, asset]
        self._names: dict[int, dict[int, str]] = {}      # boot -> name id -> name
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
        self._cache: OrderedDict = OrderedDict()       # (file, offset) -> decoded columns
        self.cache_blocks = cache_blocks
        self._pages: OrderedDict = OrderedDict()       # (file, offset, page) -> decoded page columns
        self.cache_pages = 256
        # alternate-id hashes of blocks not indexed yet (8 B per row, bounded by rows): the per-event
        # path's store check scans them; kept apart from the decoded-block cache so it neither
        # evicts query blocks nor re-reads a block per lookup while the indexer catches up
        self._building: dict[tuple, threading.Event] = {}
        self._ix_unsaved: set = set()
        self.index_ram_bytes = 4 << 30          # newest block indexes held in RAM (older: mmapped files)
        self._ix_ram: OrderedDict = OrderedDict()
        self.skipped_rows = 0
        # per-block indexes (postings by assignment + type, alternate-id hashes), built in the
        # background as blocks land and kept as memory-mapped sidecar files (see BlockIndex)
        self._ix: dict[tuple, BlockIndex] = {}
        self._ix_bad: set = set()
        self._ix_version = 0
        self._ix_tabs = None                            # (version, per-boot native lookup tables)
        self._ix_dir = os.path.join(directory, "index")
        self._ix_stop = threading.Event()
        self._ix_thread = None
        self.index_threads = index_threads or min(8, os.cpu_count() or 1)
        if index:
            os.makedirs(self._ix_dir, exist_ok=True)
            self._ix_thread = threading.Thread(target=self._index_loop, daemon=True, name=f"seg-index-{rank}")
            self._ix_thread.start()

    # ------------------------------------------------------------------ API-added events
    def _load_api_log(self):
        """Replay ``api-<rank>.log``: ``<crc32 hex> <event json>`` per line.  A torn or corrupt tail
        (a crash mid-write: the add never returned) is cut off so later appends follow good data."""
        if not os.path.exists(self._api_path):
            return
        good, events = 0, []
        with open(self._api_path, "rb") as f:
            for line in f:
                if not line.endswith(b"\n") or len(line) < 10 or line[8:9] != b" ":
                    break
                body = line[9:-1]
                try:
                    if int(line[:8], 16) != zlib.crc32(body):
                        break
                    events.append(event_from_dict(json.loads(body)))
                except ValueError:
                    break
                good += len(line)
        if good < os.path.getsize(self._api_path):
            with open(self._api_path, "r+b") as f:
                f.truncate(good)
                os.fsync(f.fileno())
        self._objects.add_events(events)

    def add_events(self, events):
        """Durable API add: the events are on disk (one fdatasync per call) before they are indexed
        and the call returns."""
        if not events:
            return events
        lines = []
        for e in events:
            body = json.dumps(e.to_dict(), separators=(",", ":")).encode()
            lines.append(b"%08x %s\n" % (zlib.crc32(body), body))
        with self._lock:
            self._api_f.write(b"".join(lines))
            self._api_f.flush()
            os.fdatasync(self._api_f.fileno())
            self._objects.add_events(events)
        return events

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
        b = int(d.get("boot", 0))
        self._asg.setdefault(b, {}).update({int(k): v for k, v in (d.get("asg") or {}).items()})
        self._names.setdefault(b, {}).update({int(k): v for k, v in (d.get("names") or {}).items()})
        self._rules.update(d.get("rules") or {})

    def add_dictionary(self, boot, asg: dict | None = None, names: dict | None = None, rules: dict | None = None):
        b = boot_id(boot)
        d = {"boot": b}
        if asg:
            d["asg"] = {int(k): list(v) for k, v in asg.items()}
        if names:
            d["names"] = {int(k): v for k, v in names.items()}
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
                  src=None) -> int:
        """Queue a sealed block for the disk; returns its token.  A replay of rows already queued
        returns the token of the block holding them (-1 once they are durable).
        ``src``: input offsets the block completes (see :meth:`SegmentStore.append`; the block must
        carry ``FLAG_COMMIT``)."""
        h = np.frombuffer((ctypes.c_uint8 * 64).from_address(ptr), np.uint8).view(HDR)[0]
        b = int(h["boot"])
        if boot is not None and boot_id(boot) != b:
            raise ValueError("dictionary boot differs from the block's")
        self.add_dictionary(b, asg, names, rules)
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
        self._ix_stop.set()
        if self._ix_thread is not None:
            self._ix_thread.join(30)
        self.seg.close()
        for f in (self._dict_f, self._api_f):
            try:
                f.close()
            except Exception:  # noqa: BLE001
                pass

    # ------------------------------------------------------------------ block indexes
    @staticmethod
    def _key(ent) -> tuple:
        return int(ent["file"]), int(ent["offset"])

    def _ix_base(self, key) -> str:
        return os.path.join(self._ix_dir, f"{key[0]}-{key[1]}")

    def _built(self, ent) -> "BlockIndex | None":
        """The block's index, built once and live as soon as it is built: the indexer threads and
        the store checks that reach a block before the indexer does share the one build in flight
        (each used to build its own: the sampled alternate-id tenant path spent as much time in the
        store checks' duplicate builds as in the indexer).  None: the block fails its checksum."""
        key = self._key(ent)
        with self._lock:
            ix = self._ix.get(key)
            if ix is not None:
                return ix
            ev = self._building.get(key)
            mine = ev is None
            if mine:
                ev = self._building[key] = threading.Event()
        if not mine:
            ev.wait()
            return self._ix.get(key)
        try:
            blk = self.seg.read_block(ent)
            if verify(blk):
                return None
            ix = BlockIndex.build(blk, int(ent["min_date"]))
            with self._lock:
                self._ix[key] = ix
                self._ix_unsaved.add(key)           # the indexer writes its files
                self._ix_version += 1
            return ix
        finally:
            with self._lock:
                self._building.pop(key, None)
            ev.set()

    def _index_one(self, ent):
        key = self._key(ent)
        ix = self._ix.get(key)
        if ix is None:
            ix = BlockIndex.load(self._ix_base(key))
            if ix is not None:
                return ix
            ix = self._built(ent)
            if ix is None:
                return None
        if key in self._ix_unsaved:
            ix.save(self._ix_base(key))
            with self._lock:
                self._ix_unsaved.discard(key)
        return ix

    def _spill_indexes(self):
        """Keep the newest block indexes in RAM (``index_ram_bytes``) and swap older ones for their
        file-backed (memory-mapped) copies: re-opening every index right after writing it held the
        indexer threads (and the interpreter) in the alternate-id tenant path."""
        for k, ix in list(self._ix.items()):
            if not isinstance(ix.pk, np.memmap) and k not in self._ix_ram and k not in self._ix_unsaved:
                self._ix_ram[k] = ix.nbytes
        total = sum(self._ix_ram.values())
        while total > self.index_ram_bytes and self._ix_ram:
            k, nb = self._ix_ram.popitem(last=False)
            total -= nb
            mm = BlockIndex.load(self._ix_base(k))
            if mm is not None and k in self._ix:
                with self._lock:        # no version bump: the search tables keep the RAM copy alive
                    self._ix[k] = mm

    def _index_loop(self):
        from concurrent.futures import ThreadPoolExecutor
        pool = ThreadPoolExecutor(self.index_threads, thread_name_prefix="seg-index")
        try:
            while not self._ix_stop.is_set():
                try:
                    ents = self.seg.index()
                except Exception:  # noqa: BLE001 -- store closing
                    break
                live = {self._key(e) for e in ents}
                for k in [k for k in self._ix if k not in live]:        # retention removed the block
                    self._ix.pop(k, None)
                    self._ix_ram.pop(k, None)
                    self._ix_unsaved.discard(k)
                    self._ix_version += 1
                    BlockIndex.remove(self._ix_base(k))
                todo = [e for e in ents if (self._key(e) not in self._ix or self._key(e) in self._ix_unsaved)
                        and self._key(e) not in self._ix_bad]
                if not todo:
                    self._ix_stop.wait(0.05)
                    continue
                # each index goes live as soon as it is built (not when the whole batch is): a
                # lagging index sends store checks to block scans
                from concurrent.futures import as_completed
                futs = {pool.submit(self._safe_index_one, e): e for e in todo[:4 * self.index_threads]}
                for f in as_completed(futs):
                    e, ix = futs[f], f.result()
                    if ix is None:
                        self._ix_bad.add(self._key(e))
                    else:
                        k = self._key(e)
                        with self._lock:
                            # an index built here went live in _built already (same object); one
                            # loaded from its files goes live now
                            fresh = k not in self._ix
                            self._ix[k] = ix
                            if fresh:
                                self._ix_version += 1
                self._spill_indexes()
        finally:
            pool.shutdown(wait=True)

    def _safe_index_one(self, ent):
        try:
            return self._index_one(ent)
        except (OSError, KeyError, ValueError):
            return None

    def index_wait(self, timeout_s: float = 60.0) -> bool:
        """Block until every block on disk is indexed (or could not be); False on timeout."""
        end = time.time() + timeout_s
        while time.time() < end:
            if all(self._key(e) in self._ix or self._key(e) in self._ix_bad for e in self.seg.index()):
                return True
            time.sleep(0.01)
        return False

    def alternate_hash_chunks(self, max_ids: int = 1 << 26, wait_s: float = 30.0):
        """The stored alternate-id hashes, newest blocks first, in chunks (numpy u64), at most
        ``max_ids``: what a restarted engine seeds its store-backed dedup filter with.  Waits up to
        ``wait_s`` for the background indexer; blocks still unindexed then are read and hashed."""
        self.index_wait(wait_s)
        left = int(max_ids)
        for e in self.seg.index()[::-1]:
            if left <= 0:
                break
            ix = self._ix.get(self._key(e))
            h = np.asarray(ix.ah if ix is not None else self._alt_index(e)[0])
            h = h[h != 0]
            if len(h):
                yield h[:left]
                left -= len(h)

    def index_stats(self) -> dict:
        ents = self.seg.index()
        return {"blocks": len(ents), "indexed": sum(self._key(e) in self._ix for e in ents),
                "index_bytes": sum(ix.nbytes for ix in list(self._ix.values()))}

    def _tables(self) -> dict:
        """Per boot: the indexed blocks (index order) and their arrays' addresses for the native
        multi-block searches; rebuilt when the set of indexed blocks changes."""
        tabs = self._ix_tabs
        ver = self._ix_version
        if tabs is not None and tabs[0] == ver:
            return tabs[1]
        by_boot: dict[int, list] = {}
        for e in self.seg.index():
            ix = self._ix.get(self._key(e))
            if ix is not None:
                by_boot.setdefault(int(e["boot"]), []).append((e, ix))
        out = {}
        P = ctypes.c_void_p
        for b, lst in by_boot.items():
            n = len(lst)
            addr = lambda a: a.ctypes.data if len(a) else 0  # noqa: E731
            out[b] = {"ents": [e for e, _ in lst], "ixs": [ix for _, ix in lst], "n": n,
                      "pk": (P * n)(*[addr(ix.pk) for _, ix in lst]), "pd": (P * n)(*[addr(ix.pd) for _, ix in lst]),
                      "ah": (P * n)(*[addr(ix.ah) for _, ix in lst]),
                      "npk": np.array([len(ix.pk) for _, ix in lst], np.int64),
                      "nah": np.array([len(ix.ah) for _, ix in lst], np.int64),
                      "base": np.array([ix.min_date for _, ix in lst], np.int64),
                      "wide": np.array([ix.wide for _, ix in lst], bool),
                      "keys": {self._key(e) for e, _ in lst}}
        self._ix_tabs = (ver, out)
        return out

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
                                 names=d.get("names"), rules=d.get("rules"), src=src)
        else:
            from .columnar import decode_batch
            d = decode_batch(payload)
            rows = d["rows"]
            n = len(rows)
            blk = encode_block(rows)
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

    @staticmethod
    def _eids(h, idx) -> np.ndarray:
        return (int(h["first_seq"]) + np.asarray(idx, np.int64)) * int(h["world"]) + int(h["rank"])

    def _alt_index(self, ent) -> tuple[np.ndarray, np.ndarray]:
        """(sorted alternate-id hashes, their rows) of a block: its index, built now (and shared with
        the indexer, ``_built``) when the background indexer has not reached the block yet."""
        ix = self._built(ent)
        if ix is None:
            raise ValueError("event block checksum mismatch")
        return ix.ah, ix.ar

    def _alt_rows(self, ent, want: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
        """(hashes, rows) of a block's rows whose alternate-id hash is in ``want`` (sorted unique)."""
        ix = self._ix.get(self._key(ent))
        ah, ar = (ix.ah, ix.ar) if ix is not None else self._alt_index(ent)
        if not len(ah):
            return np.zeros(0, np.uint64), np.zeros(0, np.int64)
        lo = np.searchsorted(ah, want, "left")
        hi = np.searchsorted(ah, want, "right")
        sel = np.nonzero(hi > lo)[0]
        if not len(sel):
            return np.zeros(0, np.uint64), np.zeros(0, np.int64)
        idx = np.concatenate([np.arange(lo[i], hi[i]) for i in sel])
        return np.asarray(ah[idx]), np.asarray(ar[idx], np.int64)

    def find_alternate_hashes(self, hashes, covered: tuple | None = None, indexed_only: bool = False) -> dict:
        """alt-id hash -> event id string for the hashes present on disk, the newest event per hash
        (store-backed dedup beyond the engine's window: ``AlternateIdDeduplicator`` asks the event
        store whether the id was ever seen).  ``covered`` = (boot, rank, sequence): that engine's
        dedup window still holds every id of its rows from ``sequence`` on, so its blocks there that
        are not indexed yet need no scan (the caller asks only about ids the window does not hold).
        ``indexed_only``: no block scans at all (binary searches of the indexed blocks only)."""
        want = np.unique(np.asarray(list(hashes), np.uint64))
        found = {}
        if not len(want):
            return found
        ents = self.seg.index()
        order: dict = {}
        best: dict[int, tuple] = {}                      # hash -> (store position, event id, boot)

        def store_pos(e) -> int:                         # built on the first hit only
            if not order:
                order.update({self._key(x): k for k, x in enumerate(ents)})
            return order.get(self._key(e), -1)

        def offer(hv, pos, eid, boot):
            cur = best.get(hv)
            if cur is None or (pos, eid) > cur[:2]:
                best[hv] = (pos, eid, boot)

        # indexed blocks: one native pass per boot over every block's sorted hashes (the newest
        # block holding each id), instead of a search per block in Python
        lib = native()
        blk, at = np.empty(len(want), np.int64), np.empty(len(want), np.int64)
        indexed = set()
        for tab in self._tables().values():
            indexed |= tab["keys"]
            lib.swseg_multi_find_u64(tab["ah"], _p(tab["nah"]), tab["n"], _p(want), len(want), _p(blk), _p(at))
            for j in np.nonzero(blk >= 0)[0].tolist():
                e = tab["ents"][int(blk[j])]
                row = int(tab["ixs"][int(blk[j])].ar[int(at[j])])
                offer(int(want[j]), store_pos(e), int(self._eids(e, [row])[0]), int(e["boot"]))
        if not indexed_only:
            for k in range(len(ents) - 1, -1, -1):       # blocks not indexed yet: scanned, newest first
                e = ents[k]
                if self._key(e) in indexed or self._ix.get(self._key(e)) is not None:
                    continue
                if covered is not None and int(e["boot"]) == covered[0] and int(e["rank"]) == covered[1] \
                        and int(e["first_seq"]) >= covered[2]:
                    continue
                hs, rows = self._alt_rows(e, want)
                if len(rows):
                    for hv, eid in zip(hs.tolist(), self._eids(e, rows).tolist()):
                        offer(int(hv), k, int(eid), int(e["boot"]))
        for hv, (_, eid, boot) in best.items():
            found[hv] = f"{boot:x}-{eid}"
        return found

    def get_event_by_alternate_id(self, alt: str):
        from ..pipeline.fleet import hash64
        ev = self._objects.get_event_by_alternate_id(alt)
        if ev is not None:
            return ev
        h = hash64(alt)
        want = np.array([h], np.uint64)
        hits = {}                                      # indexed block -> rows with the hash
        indexed = set()
        lib = native()
        for tab in self._tables().values():
            lo, hi = np.zeros(tab["n"], np.int64), np.zeros(tab["n"], np.int64)
            lib.swseg_multi_range_u64(tab["ah"], _p(tab["nah"]), tab["n"], int(h), _p(lo), _p(hi))
            for i in np.nonzero(hi > lo)[0]:
                ix = tab["ixs"][i]
                hits[self._key(tab["ents"][i])] = np.asarray(ix.ar[int(lo[i]):int(hi[i])], np.int64)
            indexed |= tab["keys"]
        for e in self.seg.index()[::-1]:               # newest first: the latest event with the id
            k = self._key(e)
            if k in indexed:
                rows = hits.get(k)
                if rows is None:
                    continue
            else:
                _, rows = self._alt_rows(e, want)
            for r in sorted(rows.tolist(), reverse=True):
                c, i = self._row_event(e, r)
                if row_strings(c, i)[0] == alt:
                    return self._materialize(c, i)
        return None

    def get_event_by_id(self, id: str):
        boot, sep, num = id.rpartition("-")
        try:
            b = int(boot, 16)
        except ValueError:
            b = None
        if not (sep and num.isdigit()) or b is None:
            return self._objects.get_event_by_id(id)
        eid = int(num)
        for e in self.seg.index():
            if int(e["boot"]) != b:
                continue
            w, r = int(e["world"]), int(e["rank"])
            if (eid - r) % w:
                continue
            row = (eid - r) // w - int(e["first_seq"])
            if 0 <= row < int(e["n_rows"]):
                c, i = self._row_event(e, row)
                return self._materialize(c, i)
        return self._objects.get_event_by_id(id)

    def list_command_responses_for_invocation(self, invocation_id, criteria=None):
        return self._objects.list_command_responses_for_invocation(invocation_id, criteria)

    def _block_hits(self, e, et: int, a: np.ndarray, c: DateRangeSearchCriteria, need: int):
        """(count, dates, rows) of a block's rows of type ``et`` whose assignment index is in ``a``
        within the date range; ``dates`` / ``rows`` hold at least the ``need`` newest of them (all of
        them when the block is not indexed)."""
        ix = self._ix.get(self._key(e))
        if ix is None or ix.wide:
            cols = self._decoded(e)
            m = (cols["etype"] == et) & np.isin(cols["asg"], a)
            if c.start_date is not None:
                m &= cols["date"] >= c.start_date
            if c.end_date is not None:
                m &= cols["date"] <= c.end_date
            idx = np.nonzero(m)[0]
            return len(idx), cols["date"][idx], idx
        keys = (a.astype(np.uint64) << np.uint64(3)) | np.uint64(et)
        keys = keys.astype(np.uint32)
        lo = np.searchsorted(ix.pk, keys, "left")
        hi = np.searchsorted(ix.pk, keys, "right")
        sel = np.nonzero(hi > lo)[0]
        if not len(sel):
            return 0, np.zeros(0, np.int64), np.zeros(0, np.int64)
        base = int(ix.min_date)
        bounded = c.start_date is not None or c.end_date is not None
        count, dates, rows = 0, [], []
        for i in sel:
            l, h = int(lo[i]), int(hi[i])
            d = np.asarray(ix.pd[l:h], np.int64) + base         # newest first within the key
            if bounded:
                # dates descend within a key: the range is one contiguous slice
                if c.end_date is not None:
                    l2 = int(np.searchsorted(-d, -c.end_date, "left"))
                else:
                    l2 = 0
                h2 = int(np.searchsorted(-d, -c.start_date, "right")) if c.start_date is not None else len(d)
                d = d[l2:h2]
                r = np.asarray(ix.pr[l + l2:l + h2], np.int64)
            else:
                r = np.asarray(ix.pr[l:h], np.int64)
            count += len(d)
            if need > 0:
                dates.append(d[:need])
                rows.append(r[:need])
        if not rows:
            return count, np.zeros(0, np.int64), np.zeros(0, np.int64)
        return count, np.concatenate(dates), np.concatenate(rows)

    def list_events(self, event_type, index, entity_ids, criteria: DateRangeSearchCriteria | None = None):
        """Events of one type for entities of an index, newest first.  Indexed blocks answer from
        their postings (assignment + type, dates descending): the total is a sum of posting-range
        lengths and only the requested page's rows are read (one page read each); blocks not
        indexed yet are decoded and scanned."""
        c = criteria or DateRangeSearchCriteria(page_size=100)
        et = _ETYPE.get(DeviceEventType(event_type))
        objs = self._objects.list_events(event_type, index, entity_ids, DateRangeSearchCriteria(
            page_size=0, start_date=c.start_date, end_date=c.end_date)).results
        if et is None:
            return SearchResults(len(objs), c.slice(objs))
        pos = _CTX[DeviceEventIndex(index)]
        want = set(entity_ids)
        with self._lock:
            asg_idx = {b: np.array(sorted(i for i, ctx in d.items() if ctx[pos] in want), np.int64)
                       for b, d in self._asg.items()}
        paged = c.page_size > 0
        need = max(1, c.page_number) * c.page_size if paged else 1 << 62
        total = len(objs)
        parts = []                     # (dates, eids, block entry, rows)
        tabs = self._tables()
        lib = native()
        d_lo = c.start_date if c.start_date is not None else -(1 << 62)
        d_hi = c.end_date if c.end_date is not None else (1 << 62)
        done = set()
        for b, a in asg_idx.items():
            tab = tabs.get(b)
            if tab is None or not len(a):
                continue
            lo, hi = np.zeros(tab["n"], np.int64), np.zeros(tab["n"], np.int64)
            for key in ((a.astype(np.uint64) << np.uint64(3)) | np.uint64(et)).astype(np.uint32).tolist():
                lib.swseg_multi_range_u32(tab["pk"], tab["pd"], _p(tab["npk"]), _p(tab["base"]), tab["n"], key,
                                          int(d_lo), int(d_hi), _p(lo), _p(hi))
                cnt = hi - lo
                cnt[tab["wide"]] = 0                       # wide blocks: scanned below
                total += int(cnt.sum())
                for i in np.nonzero(cnt > 0)[0]:
                    e, ix = tab["ents"][i], tab["ixs"][i]
                    l, h = int(lo[i]), int(min(hi[i], lo[i] + need))
                    r = np.asarray(ix.pr[l:h], np.int64)
                    parts.append((np.asarray(ix.pd[l:h], np.int64) + ix.min_date, self._eids(e, r), e, r))
            done |= {self._key(e) for e, w in zip(tab["ents"], tab["wide"]) if not w}
        for e in self.seg.index():                     # blocks not indexed (yet): decode and scan
            if self._key(e) in done:
                continue
            a = asg_idx.get(int(e["boot"]))
            if a is None or not len(a):
                continue
            if c.start_date is not None and int(e["max_date"]) < c.start_date:
                continue
            if c.end_date is not None and int(e["min_date"]) > c.end_date:
                continue
            n, d, r = self._block_hits(e, et, a, c, need)
            total += n
            if len(r):
                parts.append((d, self._eids(e, r), e, r))
        if not parts:
            return SearchResults(total, c.slice(objs))
        dates = np.concatenate([x[0] for x in parts])
        eids = np.concatenate([x[1] for x in parts])
        which = np.concatenate([np.full(len(x[0]), k, np.int32) for k, x in enumerate(parts)])
        rows = np.concatenate([x[3] for x in parts])
        order = np.lexsort((-eids, -dates))
        if objs:
            if paged:
                order = order[:need + len(objs)]
            merged = [self._materialize(*self._row_event(parts[which[o]][2], int(rows[o]))) for o in order] + objs
            merged.sort(key=lambda ev: -(ev.event_date or 0))
            return SearchResults(total, c.slice(merged))
        if paged:
            start = (max(1, c.page_number) - 1) * c.page_size
            order = order[start:start + c.page_size]
        return SearchResults(total, [self._materialize(*self._row_event(parts[which[o]][2], int(rows[o])))
                                     for o in order])

    def _materialize(self, cols: dict, i: int):
        b = cols["header"]["boot"]
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
    h = cols["header"]
    b = h["boot"]
    ctx = asg.get(int(cols["asg"][i])) or [None] * 5
    row = int(cols.get("row0", 0)) + i
    eid = (h["first_seq"] + row) * h["world"] + h["rank"]
    alt, msg, md = row_strings(cols, i)
    f = int(cols["flags"][i])
    base = dict(id=f"{b:x}-{eid}", device_assignment_id=ctx[0], device_id=ctx[1], customer_id=ctx[2],
                area_id=ctx[3], asset_id=ctx[4], event_date=int(cols["date"][i]), received_date=h["recv_ms"],
                alternate_id=alt, metadata=md)
    et = int(cols["etype"][i])
    nid = int(cols["name"][i])
    name = names.get(nid, "") if nid != NO_NAME else ""
    if et == EV_MEASUREMENT:
        return DeviceMeasurement(name=name, value=float(cols["v0"][i]), **base)
    if et == EV_LOCATION:
        return DeviceLocation(latitude=float(cols["v0"][i]), longitude=float(cols["v1"][i]),
                              elevation=float(cols["v2"][i]) if f & SEGF_HAS_ELEV else None, **base)
    if et == EV_ALERT:
        gen = bool(f & SEGF_GEN)
        return DeviceAlert(source=AlertSource.System if gen else AlertSource.Device,
                           level=_LEVELS[min(int(cols["level"][i]), 3)], type=name,
                           message=(rules.get(name) or "") if gen else msg, **base)
    # the engine's state changes are its presence scan (DevicePresenceManager.java:110-200)
    return DeviceStateChange(attribute="presence", type="presence", previous_state="PRESENT",
                             new_state="NOT_PRESENT", **base)
