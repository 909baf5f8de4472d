"""Events added through the API (REST / RPC adds, command invocations and responses, rule alerts) as
rows of the same durable, indexed blocks the engine writes (``persistence/segments.py``).

The reference writes every add to the one indexed Mongo collection, through a buffer
(``MongoDeviceEventManagement.java:191-405``, ``DeviceEventBuffer.java:99-135``).  Here an add is
durable before it returns -- one fdatasync'd line in a short write-ahead log (group-committed
across concurrent callers) -- and visible at once from the store's in-memory tail; the tail is
encoded into a block with its index trailer (``swseg_encode`` + ``swseg_index_append`` on the host:
the format the MI355X builds) every ``flush_events`` events or ``flush_s`` seconds, appended to the
segment store under the same commit discipline, and the log is cut back to what is not yet in a
block.  So the store's memory and its restart time are bounded by the tail, not by history.

Row encoding (one block row per event; ``swseg.h``):
  * Measurement: name -> name column (per-boot dictionary), value -> v0;
  * Location: latitude / longitude -> v0 / v1, elevation (flagged when sent);
  * Alert: type -> name, level, message -> message heap; source System -> ``SEGF_SYS``;
  * CommandInvocation / CommandResponse / StateChange: their type-specific fields as a JSON object
    in the metadata span (``SEGF_JSON``; the event's metadata rides inside it);
  * every row: assignment -> the boot's assignment dictionary (assignment, device, customer, area,
    asset tokens; customer / area / asset also get the context ids the trailers index), alternate
    id -> the id heap (indexed), metadata -> protobuf ``Metadata`` entries (as devices send them).

Event ids are the store's own: ``<api boot hex>-<sequence>``, assigned at add time (the blocks' row
sequence), like engine events."""
from __future__ import annotations

import json

import numpy as np

from ..models.columnar import (EV_ALERT, EV_COMMAND_INVOCATION, EV_COMMAND_RESPONSE, EV_LOCATION, EV_MEASUREMENT,
                               EV_STATE_CHANGE, EVENT_REC, NO_NAME, OUT_REC, SR_ALT, SR_META, STR_REF)
from ..models.domain import (ALERT_LEVEL_INDEX, AlertSource, DeviceAlert, DeviceCommandInvocation,
                             DeviceCommandResponse, DeviceEventType, DeviceLocation, DeviceMeasurement,
                             DeviceStateChange)

SW_F_HAS_ELEVATION, SW_F_SYS_ALERT, SW_F_JSON = 0x8, 0x10, 0x20
_META_FIELD = {EV_MEASUREMENT: 4, EV_LOCATION: 6, EV_ALERT: 5}
_ETYPE = {DeviceEventType.Measurement: EV_MEASUREMENT, DeviceEventType.Location: EV_LOCATION,
          DeviceEventType.Alert: EV_ALERT, DeviceEventType.CommandInvocation: EV_COMMAND_INVOCATION,
          DeviceEventType.CommandResponse: EV_COMMAND_RESPONSE, DeviceEventType.StateChange: EV_STATE_CHANGE}
MAX_STR = 0xFFFF                     # string spans are u16 in the block format


def _varint(n: int) -> bytes:
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def metadata_wire(md: dict, field: int) -> bytes:
    """Metadata entries as protobuf ``Model.Metadata {name = 1; value = 2}`` fields ``field`` (what
    :func:`segments.parse_metadata` reads back, and what devices send)."""
    out = bytearray()
    for k, v in md.items():
        kb, vb = str(k).encode(), ("" if v is None else str(v)).encode()
        ent = b"\x0a" + _varint(len(kb)) + kb + b"\x12" + _varint(len(vb)) + vb
        out += _varint((field << 3) | 2) + _varint(len(ent)) + ent
    return bytes(out)


def json_fields(e) -> dict:
    """Type-specific fields of a JSON-encoded row (and the event's metadata under "m")."""
    d = {}
    if isinstance(e, DeviceCommandInvocation):
        d = {"i": getattr(e.initiator, "value", e.initiator), "ii": e.initiator_id,
             "t": getattr(e.target, "value", e.target), "ti": e.target_id, "dc": e.device_command_id,
             "ct": e.command_token, "pv": e.parameter_values or {}}
    elif isinstance(e, DeviceCommandResponse):
        d = {"o": e.originating_event_id, "r": e.response_event_id, "s": e.response}
    elif isinstance(e, DeviceStateChange):
        d = {"a": e.attribute, "ty": e.type, "p": e.previous_state, "n": e.new_state}
    if e.metadata:
        d["m"] = e.metadata
    return {k: v for k, v in d.items() if v is not None}


def event_from_json_row(etype: int, fields: dict, base: dict):
    """The event of a JSON-encoded row (:func:`json_fields`) with the common fields ``base``."""
    base = dict(base, metadata=fields.get("m") or {})
    if etype == EV_COMMAND_INVOCATION:
        return DeviceCommandInvocation(initiator=fields.get("i", "REST"), initiator_id=fields.get("ii"),
                                       target=fields.get("t", "Assignment"), target_id=fields.get("ti"),
                                       device_command_id=fields.get("dc"), command_token=fields.get("ct"),
                                       parameter_values=fields.get("pv") or {}, **base)
    if etype == EV_COMMAND_RESPONSE:
        return DeviceCommandResponse(originating_event_id=fields.get("o"), response_event_id=fields.get("r"),
                                     response=fields.get("s"), **base)
    return DeviceStateChange(attribute=fields.get("a", ""), type=fields.get("ty", ""),
                             previous_state=fields.get("p"), new_state=fields.get("n"), **base)


class ApiDictionary:
    """The API boot's dictionaries, as the store keeps them (``DurableEventStore._asg`` / ``_names`` /
    ``_ctx`` for that boot), with reverse maps for encoding; ``take_delta`` hands out what new rows
    added (the store writes it to its dictionary log before the block)."""

    def __init__(self, asg: dict, names: dict, ctx: dict):
        self.asg_of = {tuple(v): int(k) for k, v in asg.items()}
        self.name_of = {v: int(k) for k, v in names.items()}
        self.ctx_of = {int(d): dict(m) for d, m in ctx.items()}
        self.next_asg = max(asg, default=-1) + 1
        self.next_name = max(names, default=-1) + 1
        self.d_asg: dict = {}
        self.d_names: dict = {}
        self.d_ctx: dict = {}

    def asg(self, e) -> int:
        key = (e.device_assignment_id, e.device_id, e.customer_id, e.area_id, e.asset_id)
        i = self.asg_of.get(key)
        if i is None:
            i = self.asg_of[key] = self.next_asg
            self.next_asg += 1
            self.d_asg[i] = list(key)
            for dim, tok in enumerate(key[2:]):
                if tok is not None and tok not in self.ctx_of.setdefault(dim, {}):
                    cid = len(self.ctx_of[dim])
                    self.ctx_of[dim][tok] = cid
                    self.d_ctx.setdefault(dim, {})[tok] = cid
        return i

    def name(self, s: str) -> int:
        i = self.name_of.get(s)
        if i is None:
            if self.next_name >= NO_NAME:
                return NO_NAME                        # dictionary full: the row keeps no name
            i = self.name_of[s] = self.next_name
            self.next_name += 1
            self.d_names[i] = s
        return i

    def ctx_table(self) -> np.ndarray:
        """int32 [assignments, 4]: (assignment, customer, area, asset context ids; -1 none)."""
        n = self.next_asg
        tab = np.full((max(n, 1), 4), -1, np.int32)
        tab[:, 0] = np.arange(len(tab))
        for key, i in self.asg_of.items():
            for dim, tok in enumerate(key[2:]):
                if tok is not None:
                    tab[i, 1 + dim] = self.ctx_of.get(dim, {}).get(tok, -1)
        return tab

    def take_delta(self) -> tuple[dict, dict, dict]:
        d = (self.d_asg, self.d_names, self.d_ctx)
        self.d_asg, self.d_names, self.d_ctx = {}, {}, {}
        return d


def row_limit_error(e) -> str | None:
    """Why ``e`` cannot be one block row, or None.  String spans are u16 in the block format: the
    alternate id, an alert's message and the metadata (or JSON fields) span each hold <= 65535 bytes.
    ``DurableEventStore.add_events`` checks this before the event reaches its write-ahead log, so an
    add is refused up front instead of failing every later flush of the API tail (nothing is ever
    truncated: a cut alternate id would also break its dedup)."""
    et = _ETYPE.get(DeviceEventType(e.event_type))
    if et is None:
        return f"event type {e.event_type} cannot be stored"
    if e.alternate_id and len(e.alternate_id.encode()) > MAX_STR:
        return f"alternate id longer than {MAX_STR} bytes"
    if et == EV_ALERT and e.message and len(e.message.encode()) > MAX_STR:
        return f"alert message longer than {MAX_STR} bytes"
    if et in (EV_MEASUREMENT, EV_LOCATION, EV_ALERT):
        meta = metadata_wire(e.metadata, _META_FIELD[et]) if e.metadata else b""
    else:
        meta = json.dumps(json_fields(e), separators=(",", ":")).encode()
    if len(meta) > MAX_STR:
        return f"event fields / metadata too large for a block row ({len(meta)} > {MAX_STR} bytes)"
    return None


def encode_events(events, dic: ApiDictionary):
    """API events -> (OUT_REC rows, EVENT_REC records, STR_REF spans, string bytes) for
    :func:`segments.encode_block`, in the given order."""
    n = len(events)
    rows = np.zeros(n, OUT_REC)
    recs = np.zeros(n, EVENT_REC)
    spans = np.zeros(n, STR_REF)
    heap = bytearray()
    recs["fp_lo"] = 1                                 # not engine-generated: strings are kept
    for i, e in enumerate(events):
        et = _ETYPE[DeviceEventType(e.event_type)]
        r, x, s = rows[i], recs[i], spans[i]
        r["event_date"] = int(e.event_date or 0)
        r["assignment"] = dic.asg(e)
        r["etype"] = et
        r["name_id"] = NO_NAME
        x["etype"] = et
        x["event_date"] = int(e.event_date or 0)
        flags = 0
        md = e.metadata or {}
        meta = b""
        if et == EV_MEASUREMENT:
            r["name_id"] = dic.name(e.name or "")
            r["v0"] = float(e.value or 0.0)
        elif et == EV_LOCATION:
            r["v0"], r["v1"] = float(e.latitude or 0.0), float(e.longitude or 0.0)
            if e.elevation is not None:
                x["v2"] = float(e.elevation)
                flags |= SW_F_HAS_ELEVATION
        elif et == EV_ALERT:
            r["name_id"] = dic.name(e.type or "")
            r["level"] = ALERT_LEVEL_INDEX.get(e.level, 0) if not isinstance(e.level, int) else e.level
            if AlertSource(e.source) == AlertSource.System:
                flags |= SW_F_SYS_ALERT
            mb = (e.message or "").encode()
            if len(mb) > MAX_STR:
                raise ValueError(f"alert message longer than {MAX_STR} bytes")
            if mb:
                x["aux2_off"], x["aux2_len"] = len(heap), len(mb)
                heap += mb
        else:
            flags |= SW_F_JSON
            meta = json.dumps(json_fields(e), separators=(",", ":")).encode()
        if md and not (flags & SW_F_JSON):
            meta = metadata_wire(md, _META_FIELD[et])
        x["flags"] = flags
        has = 0
        if e.alternate_id:
            ab = e.alternate_id.encode()
            if len(ab) > MAX_STR:
                raise ValueError(f"alternate id longer than {MAX_STR} bytes")
            s["alt_off"], s["alt_len"] = len(heap), len(ab)
            heap += ab
            has |= SR_ALT
        if meta:
            if len(meta) > MAX_STR:
                raise ValueError(f"event fields too large for a block row ({len(meta)} bytes)")
            s["meta_off"], s["meta_len"] = len(heap), len(meta)
            heap += meta
            has |= SR_META
        s["has"] = has
    return rows, recs, spans, np.frombuffer(bytes(heap) + b"\0" * 64, np.uint8)
