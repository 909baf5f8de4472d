"""Columnar / fixed-width record layouts shared by the host runtime and the gfx950 kernels.

These numpy dtypes mirror the C structs in ``csrc/include/swtypes.h`` and
``csrc/include/swengine.h`` byte for byte (``tests/test_columnar.py`` checks
them against ``sw_abi_sizes`` and field offsets).
"""
from __future__ import annotations

import numpy as np

# Event types (GDeviceEventType in the reference's device-event-model.proto).
EV_MEASUREMENT = 0
EV_LOCATION = 1
EV_ALERT = 2
EV_COMMAND_INVOCATION = 3
EV_COMMAND_RESPONSE = 4
EV_STATE_CHANGE = 5
EV_REGISTRATION = 16
EV_ACK = 17
EV_STREAM_CREATE = 18
EV_STREAM_DATA = 19
EV_STREAM_DATA_REQUEST = 20
EV_DECODE_ERROR = 255

# Validation status (InboundPayloadProcessingLogic outcomes).
ST_OK = 0
ST_UNREGISTERED = 1
ST_UNASSIGNED = 2
ST_DUPLICATE = 3
ST_DECODE_ERROR = 4
ST_CONTROL = 5
ST_RECHECK = 6          # id new to the dedup window, maybe stored before: host checks the store

F_HAS_UPDATE_STATE = 0x1
F_UPDATE_STATE = 0x2
F_HAS_DATE = 0x4
F_HAS_ELEVATION = 0x8
F_SETTLED = 0x40       # store-backed dedup settled on the host: the filter skips the record

EVENT_REC = np.dtype([
    ("fp_lo", "<u8"), ("fp_hi", "<u8"), ("event_date", "<i8"), ("name_hash", "<u8"),
    ("v0", "<f8"), ("v1", "<f8"), ("v2", "<f8"), ("alt_hash", "<u8"),
    ("aux_off", "<u4"), ("aux2_off", "<u4"), ("aux_len", "<u2"), ("aux2_len", "<u2"),
    ("etype", "u1"), ("flags", "u1"), ("src_rank", "u1"), ("level", "u1"),
], align=True)
assert EVENT_REC.itemsize == 80

# String refs of a decoded event (SwStrRef, csrc/include/swtypes.h): where its alternate id and
# metadata span sit in the raw batch, and its measurement index (alternate id "<alt>:<k>").
STR_REF = np.dtype([("alt_off", "<u4"), ("meta_off", "<u4"), ("alt_len", "<u2"), ("meta_len", "<u2"),
                    ("k", "<u2"), ("has", "u1"), ("pad", "u1")], align=True)
assert STR_REF.itemsize == 16
SR_ALT, SR_META, SR_MULTI = 0x1, 0x2, 0x4
EV_OVERSIZE = 21

# Exchange form (SwWireRec, csrc/include/swtypes.h): lossless 64-byte packing of EVENT_REC.
WIRE_REC = np.dtype([
    ("fp_lo", "<u8"), ("fp_hi", "<u8"), ("event_date", "<i8"), ("w0", "<u8"), ("w1", "<u8"), ("w2", "<u8"),
    ("alt_hash", "<u8"), ("aux_off", "<u4"), ("aux_len", "<u2"), ("etype", "u1"), ("flags", "u1"),
], align=True)
assert WIRE_REC.itemsize == 64


def wire_pack(r: np.ndarray) -> np.ndarray:
    """EVENT_REC -> WIRE_REC (same rule as ``sw_wire_pack``)."""
    w = np.zeros(len(r), WIRE_REC)
    for k in ("fp_lo", "fp_hi", "event_date", "alt_hash", "aux_off", "aux_len", "etype", "flags"):
        w[k] = r[k]
    loc = r["etype"] == 1
    val = (r["etype"] == 0) | loc
    w["w0"] = np.where(loc, r["v2"].view(np.uint64), r["name_hash"])
    aux2 = (r["aux2_off"].astype(np.uint64) | (r["aux2_len"].astype(np.uint64) << np.uint64(32)) |
            (r["level"].astype(np.uint64) << np.uint64(48)))
    w["w1"] = np.where(val, r["v0"].view(np.uint64), aux2)
    w["w2"] = r["v1"].view(np.uint64)
    return w


def wire_unpack(w: np.ndarray, src_rank: int) -> np.ndarray:
    """WIRE_REC -> EVENT_REC (``sw_wire_unpack``); ``src_rank`` = the slab the records came from."""
    r = np.zeros(len(w), EVENT_REC)
    for k in ("fp_lo", "fp_hi", "event_date", "alt_hash", "aux_off", "aux_len", "etype", "flags"):
        r[k] = w[k]
    loc = w["etype"] == 1
    val = (w["etype"] == 0) | loc
    r["name_hash"] = np.where(loc, np.uint64(0), w["w0"])
    r["v2"] = np.where(loc, w["w0"], np.uint64(0)).view(np.float64)
    r["v0"] = np.where(val, w["w1"], np.uint64(0)).view(np.float64)
    r["v1"] = w["w2"].view(np.float64)
    aux = np.where(val, np.uint64(0), w["w1"])
    r["aux2_off"] = (aux & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    r["aux2_len"] = ((aux >> np.uint64(32)) & np.uint64(0xFFFF)).astype(np.uint16)
    r["level"] = ((aux >> np.uint64(48)) & np.uint64(0xFF)).astype(np.uint8)
    r["src_rank"] = src_rank
    return r


OUT_REC = np.dtype([
    ("event_date", "<i8"), ("v0", "<f8"), ("v1", "<f8"), ("assignment", "<i4"), ("name_id", "<u2"),
    ("etype", "u1"), ("level", "u1"),
])
OUT_REC_SIZE = 32
assert OUT_REC.itemsize == OUT_REC_SIZE
NO_NAME = 0xFFFF

NAME_REF = np.dtype([("hash", "<u8"), ("off", "<u4"), ("len", "<u2"), ("src_rank", "u1"), ("etype", "u1")])
assert NAME_REF.itemsize == 16

REG_SLOT = np.dtype([("lo", "<u8"), ("hi", "<u8"), ("dev", "<i4"), ("asg", "<i4"), ("pad", "<u8")])
assert REG_SLOT.itemsize == 32
ASG_STATE = np.dtype([("last", "<u8"), ("missing", "<u8"), ("loc_date", "<u8"), ("loc_eid1", "<u8")])
MS_SLOT = np.dtype([("key", "<u8"), ("date", "<u8"), ("eid1", "<u8"), ("pad", "<u8")])

ZONE_TEST = np.dtype([("zone", "<i4"), ("condition", "<i4"), ("alert_name_id", "<i4"), ("level", "<i4")])

# Stats slots (SW_STAT_* in swengine.h).
N_STATS = 24            # SW_N_STATS (csrc/include/swengine.h): slots of the stats arrays
STAT_NAMES = [
    "messages", "events", "persisted", "unregistered", "unassigned", "duplicates", "decode_errors",
    "control", "rule_alerts", "presence_events", "shuffle_overflow", "new_names", "state_overflow",
    "shuffle_deferred", "dedup_overflow", "dedup_rotations", "dedup_rechecks",
]

# Alert levels (GAlertLevel) and sources.
ALERT_LEVELS = ["Info", "Warning", "Error", "Critical"]

EVENT_TYPE_NAMES = {
    EV_MEASUREMENT: "Measurement", EV_LOCATION: "Location", EV_ALERT: "Alert",
    EV_COMMAND_INVOCATION: "CommandInvocation", EV_COMMAND_RESPONSE: "CommandResponse",
    EV_STATE_CHANGE: "StateChange",
}
