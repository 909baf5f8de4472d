"""Where a durable block's bytes go, per event: page headers, each column's packed bits and double
exceptions, the string heap, and the index trailer's sections -- for a bench-shaped step (bench.py
fleet: 1M devices, alternate ids, 0.5% unregistered, 10% metadata) encoded by the C++ encoder (the
MI355X encoder's bytes are identical, tests/test_gpu_segments.py).  Prints one JSON line."""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

COLS = ["etype", "level", "date", "asg", "name", "mxv", "lat", "lon", "elev", "flags", "altk", "altlen",
        "altnum", "msglen", "metalen"]


def breakdown(blk: np.ndarray) -> dict:
    from sitewhere_amd.persistence import segments as sg
    hdr = blk[:64].view(np.uint32)
    n_rows, n_pages = int(hdr[2]), int(hdr[3])
    poff = blk[64:64 + 4 * (n_pages + 1)].view(np.uint32)
    out = {"rows": n_rows, "pages": n_pages, "block_header": 64 + 4 * (n_pages + 1)}
    col = dict.fromkeys(COLS, 0)
    exc = dict.fromkeys(COLS, 0)
    heap = hdrs = pad = 0
    for p in range(n_pages):
        base = int(poff[p])
        ph = blk[base:base + sg.PAGE_HDR]
        pbytes = int(ph[4:8].view(np.uint32)[0])
        heap_off, heap_bytes = (int(x) for x in ph[16:24].view(np.uint32))
        hdrs += sg.PAGE_HDR
        used = sg.PAGE_HDR + heap_bytes
        heap += heap_bytes
        for c in range(len(COLS)):
            o = 40 + 24 * c
            cnt = int(ph[o + 12:o + 14].view(np.uint16)[0])
            nexc = int(ph[o + 14:o + 16].view(np.uint16)[0])
            bits = int(ph[o + 16])
            words = (cnt * bits + 63) // 64
            col[COLS[c]] += 8 * words
            e = (2 * nexc + 7) // 8 * 8 + 8 * nexc if nexc else 0
            exc[COLS[c]] += e
            used += 8 * words + e
        pad += pbytes - used
    tr = sg.trailer_offset(blk)
    end = int(blk[16:24].view(np.uint64)[0])
    out.update({"page_headers": hdrs, "heap": heap, "page_padding": pad,
                "columns": {k: v for k, v in col.items() if v}, "exceptions": {k: v for k, v in exc.items() if v},
                "trailer": end - tr if tr > 0 else 0, "bytes": end})
    if tr > 0:
        th = blk[tr:tr + 112]
        u32 = th.view(np.uint32)
        n_alt, off_pages, off_dir, off_alt = int(u32[9]), int(u32[10]), int(u32[11]), int(u32[12])
        off_keys = [int(x) for x in u32[13:16]]
        out["trailer_sections"] = {"header+pages": off_dir, "alt_dir": off_alt - off_dir,
                                   "alt_entries": off_keys[0] - off_alt, "context_keys_heads": end - tr - off_keys[0],
                                   "n_alt": n_alt}
    per = {k: round(v / max(1, n_rows), 3) for k, v in out.items() if isinstance(v, int) and k not in ("rows", "pages")}
    per["columns"] = {k: round(v / n_rows, 3) for k, v in out["columns"].items()}
    per["exceptions"] = {k: round(v / n_rows, 3) for k, v in out["exceptions"].items()}
    if "trailer_sections" in out:
        per["trailer_sections"] = {k: round(v / n_rows, 3) for k, v in out["trailer_sections"].items() if k != "n_alt"}
    out["per_row"] = per
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--msgs", type=int, default=1 << 20)
    ap.add_argument("--devices", type=int, default=1 << 20)
    a = ap.parse_args()
    from sitewhere_amd.pipeline.config import EngineConfig
    from sitewhere_amd.pipeline.fleet import FleetSpec, fingerprints, gen_payloads, gen_tokens
    from sitewhere_amd.pipeline.native_engine import NativeCpuEngine
    cfg = EngineConfig(max_msgs=a.msgs, rec_cap=a.msgs + 4096, gen_cap=a.msgs // 2, max_devices=a.devices + 1024,
                       max_assignments=a.devices + 1024, store_cap=1 << 21, dedup_slots=1 << 22, name_slots=1 << 12,
                       state_slots=1 << 23)
    e = NativeCpuEngine(cfg)
    heap, offs = gen_tokens("dev-", 0, a.devices)
    lo, hi = fingerprints(heap, offs)
    dev = e.register_devices(lo, hi)
    e.set_assignments(dev, dev, customer=dev % 97, area=dev % 31, asset=dev % 1009)
    spec = FleetSpec(prefix="dev-", n_devices=a.devices, p_location=0.25, p_alert=0.05, p_unregistered=0.005,
                     mx_per_msg=1, n_names=16, with_alternate_id=True, lat0=33.0, lon0=-85.0, span_deg=2.0,
                     p_register=0.0005, p_ack=0.0005, p_meta=0.1)
    raw, o = gen_payloads(spec, a.msgs, 1_700_000_000_000, seed=3)
    raw = np.concatenate([raw, np.zeros(64, np.uint8)])
    res = e.step(raw, o, 1_700_000_060_000, presence=False)
    blk = e.encode_block(1_700_000_060_000, res, boot=1)
    out = breakdown(np.asarray(blk))
    sp, pr = res.pspans, res.prec
    n = max(1, len(pr))
    out["per_row"]["heap_parts"] = {
        "metadata": round(float(np.where(sp["has"] & 2, sp["meta_len"], 0).sum()) / n, 3),
        "alert_messages": round(float(np.where(pr["etype"] == 2, pr["aux2_len"], 0).sum()) / n, 3)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
