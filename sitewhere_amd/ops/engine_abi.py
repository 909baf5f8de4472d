"""ctypes mirror of ``SwEngineArgs`` (csrc/include/swengine.h).

Every field is 8 bytes; the order below must match the header exactly.
``tests/test_columnar.py`` compares ``ctypes.sizeof(SwEngineArgs)`` with the
library's own ``sizeof`` (``sw_abi_sizes``).
"""
from __future__ import annotations

import ctypes

P = ctypes.c_void_p
I = ctypes.c_int64
U = ctypes.c_uint64

FIELDS = [
    # batch input
    ("raw", P), ("msg_off", P), ("n_msgs", I), ("now_ms", I), ("rank", I), ("world", I), ("batch_seq", I),
    # decode
    ("msg_cnt", P), ("msg_evoff", P), ("scan_tmp", P), ("scan_tmp_len", I),
    ("recs", P), ("rec_cap", I), ("n_recs", P),
    ("seen_key", P), ("seen_mask", I), ("new_names", P), ("n_new_names", P), ("names_cap", I),
    # shuffle
    ("send", P), ("recv", P), ("shuf_cap", I), ("send_cnt", P), ("recv_cnt", P), ("part_tmp", P),
    ("part_tmp_len", I), ("overflow", P),
    # validated batch
    ("work", P), ("n_work", P), ("status", P), ("ev_dev", P), ("ev_asg", P),
    ("ok_idx", P), ("n_ok", P), ("rej_idx", P), ("n_rej", P), ("cmp_tmp", P),
    # registry
    ("reg", P), ("reg_mask", I), ("asg_ctx", P), ("asg_active", P), ("n_asg", I),
    # dedup
    ("dd_key", P), ("dd_seq", P), ("dd_mask", I), ("seq_base", P),
    # names intern
    ("nm_key", P), ("nm_id", P), ("nm_first", P), ("nm_mask", I), ("nm_counter", P),
    # state
    ("st", P), ("ms", P), ("ms_mask", I),
    # store
    ("store_cap", I), ("store_cursor", P), ("step_cursor0", P),
    ("s_etype", P), ("s_level", P), ("s_date", P), ("s_recv", P), ("s_dev", P), ("s_asg", P),
    ("s_cust", P), ("s_area", P), ("s_asset", P), ("s_name", P), ("s_v0", P), ("s_v1", P), ("s_v2", P),
    ("s_alt", P), ("s_aux", P), ("s_batch", P),
    # outbound
    ("out", P), ("n_out", P),
    # rules
    ("zone_vtx", P), ("zone_off", P), ("zone_bbox", P), ("n_zones", I), ("tests", P), ("n_tests", I),
    ("test_name_hash", P), ("zmask", P), ("ztile", P),
    ("gen", P), ("gen_dev", P), ("gen_asg", P), ("n_gen", P), ("gen_cap", I),
    # presence
    ("presence_missing_ms", I), ("presence_name_hash", U),
    # stats
    ("stats", P),
    # per-step params (device SwStepParams, written in-stream each step)
    ("sp", P),
    # shuffle spill (records deferred to the next step's exchange)
    ("carry", P), ("n_carry", P), ("spill", P), ("n_spill", P), ("carry_cap", I),
    # rules, host-side sizes
    ("n_zone_vtx", I),
    # state merge scratch
    ("ev_slot", P),
    ("dd_meta", P),
    # string refs of the decoded records (SwStrRef, read by the durable-block encoder)
    ("spans", P),
    # store-backed dedup filter (generational fingerprint tables, swtypes.h SW_FF_*; null = off)
    ("dd_ff", P), ("dd_ff_bmask", I), ("dd_ff_gens", I), ("dd_ff_meta", P),
    # string exchange (world > 1): per-destination byte slabs + refs beside the record slabs
    ("send_str", P), ("send_str_cnt", P), ("send_spans", P), ("recv_str", P), ("recv_str_cnt", P),
    ("recv_spans", P), ("work_str", P), ("work_spans", P), ("str_cap", I), ("str_drops", P),
    # re-key destination of each partition input
    ("part_owner", P),
    # persist clustering by assignment (radix-sort buffers, key bits; 0 = arrival order)
    ("cl_keys", P), ("cl_vals", P), ("cl_hist", P), ("cl_bits", I),
    # lossless re-key: per-input string bytes, per-tile byte matrix, cut metadata, carry string heaps
    ("part_len", P), ("part_bytes", P), ("part_meta", P), ("carry_spans", P), ("carry_str", P),
    ("spill_spans", P), ("spill_str", P), ("n_spill_str", P), ("carry_str_cap", I),
]


class SwEngineArgs(ctypes.Structure):
    _fields_ = FIELDS


def abi_sizes(lib) -> dict:
    buf = (ctypes.c_int64 * 10)()
    lib.sw_abi_sizes(ctypes.cast(buf, ctypes.c_void_p))
    return {"event_rec": buf[0], "out_rec": buf[1], "engine_args": buf[2], "name_ref": buf[3], "zone_test": buf[4],
            "reg_slot": buf[5], "asg_state": buf[6], "ms_slot": buf[7], "wire_rec": buf[8],
            "str_ref": buf[9]}
