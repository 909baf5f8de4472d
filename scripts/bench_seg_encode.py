"""Microbenchmark of the MI355X durable-block encoder (``k_seg_encode``) alone: one step's persisted
rows (a generated fleet decoded on the host: alternate ids, metadata, alert messages, locations;
rule / presence rows after them), encoder aux built once by ``k_seg_aux``, then ``--reps`` encodes
timed with HIP events.  Prints one JSON line (mean / min us per encode, rows, block bytes).

    python scripts/bench_seg_encode.py --n 1048576 --reps 20 [--no-strings]"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--no-strings", action="store_true")
    ap.add_argument("--stamps", action="store_true", help="also report per-page phase times (s_memrealtime)")
    ap.add_argument("--lib", default=None, help="an encoder variant (swseg.hip built with other -DSW_SEG_* "
                    "geometry); its blocks must equal the built-in encoder's byte for byte")
    a = ap.parse_args()
    import torch

    from sitewhere_amd._native import gpu
    from sitewhere_amd.models.columnar import EVENT_REC, OUT_REC, STR_REF
    from sitewhere_amd.persistence.segments import PAGE_ROWS, max_block_bytes, max_string_bytes
    from tests.test_segments import synth_rows
    lib = gpu()
    rows, recs, spans, raw = synth_rows(a.n, seed=7, strings=not a.no_strings)
    n = len(rows)
    dev = (recs["fp_lo"] != 0) | (recs["fp_hi"] != 0)
    n_ok = int(dev.sum())
    d = torch.device("cuda", 0)

    def t(x):
        return torch.from_numpy(np.ascontiguousarray(x).view(np.uint8).reshape(-1).copy()).to(d)
    work_t = t(recs[:n_ok] if n_ok else np.zeros(1, EVENT_REC))
    wsp_t = t(spans[:n_ok] if n_ok else np.zeros(1, STR_REF))
    gen_t = t(recs[n_ok:] if n > n_ok else np.zeros(1, EVENT_REC))
    okidx = torch.arange(max(n_ok, 1), dtype=torch.int32, device=d)
    nok = torch.tensor([n_ok], dtype=torch.int32, device=d)
    rows_t = t(np.ascontiguousarray(rows, OUT_REC))
    raw_t = t(np.concatenate([raw, np.zeros(64, np.uint8)]))
    cursor = torch.tensor([n, 0], dtype=torch.int64, device=d)
    cap = max_block_bytes(n, max_string_bytes(n, len(raw)))
    pages = -(-n // PAGE_ROWS)
    blk = torch.zeros(cap, dtype=torch.uint8, device=d)
    state = torch.zeros(pages + 8, dtype=torch.int64, device=d)
    aux = torch.zeros(n * 32, dtype=torch.uint8, device=d)
    s = torch.cuda.current_stream(d)
    P = ctypes.c_void_p
    assert lib.sw_seg_aux(P(work_t.data_ptr()), P(okidx.data_ptr()), P(nok.data_ptr()), P(gen_t.data_ptr()),
                          P(wsp_t.data_ptr()), len(raw), P(cursor.data_ptr()), P(aux.data_ptr()), n,
                          P(s.cuda_stream)) == 0
    ref_block = None
    if a.lib:
        # the built-in encoder's block, then time the variant
        assert lib.sw_seg_encode(P(rows_t.data_ptr()), P(aux.data_ptr()), P(raw_t.data_ptr()), P(cursor.data_ptr()),
                                 P(blk.data_ptr()), cap, P(state.data_ptr()), pages, P(s.cuda_stream)) == 0
        s.synchronize()
        nb0 = int(state[pages + 1].item())
        ref_block = blk[:nb0].cpu().numpy().copy()
        from ctypes import c_int32, c_int64
        var = ctypes.CDLL(os.path.abspath(a.lib))
        var.sw_seg_encode.restype = c_int32
        var.sw_seg_encode.argtypes = [P, P, P, P, P, c_int64, P, c_int64, P]
        var.sw_seg_encode_stamped.restype = c_int32
        var.sw_seg_encode_stamped.argtypes = [P, P, P, P, P, c_int64, P, c_int64, P, P]
        lib = var
    times = []
    for r in range(a.reps + 2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        assert lib.sw_seg_encode(P(rows_t.data_ptr()), P(aux.data_ptr()), P(raw_t.data_ptr()), P(cursor.data_ptr()),
                                 P(blk.data_ptr()), cap, P(state.data_ptr()), pages, P(s.cuda_stream)) == 0
        e1.record(s)
        s.synchronize()
        if r >= 2:
            times.append(1000.0 * e0.elapsed_time(e1))
    nb, err, _ = (int(x) for x in state[pages + 1:pages + 4].cpu().numpy())
    assert err == 0, err
    if ref_block is not None:
        assert nb == len(ref_block) and np.array_equal(blk[:nb].cpu().numpy(), ref_block), "variant block differs"
    phases = None
    if a.stamps:
        # one more encode with per-page phase stamps (s_memrealtime, 100 MHz = 10 ns ticks)
        st = torch.zeros(pages * 16, dtype=torch.int64, device=d)
        assert lib.sw_seg_encode_stamped(P(rows_t.data_ptr()), P(aux.data_ptr()), P(raw_t.data_ptr()),
                                         P(cursor.data_ptr()), P(blk.data_ptr()), cap, P(state.data_ptr()), pages,
                                         P(st.data_ptr()), P(s.cuda_stream)) == 0
        s.synchronize()
        x = st.cpu().numpy().reshape(pages, 16)[:, :11].astype(np.int64) * 10      # ns
        t0 = x[:, 0].min()
        names = ["load", "r1", "r2", "r3", "layout", "lookback", "-", "pairs", "heap", "hdr+cs"]
        dur = np.diff(x, axis=1)
        phases = {nm: {"p50_us": round(float(np.median(dur[:, i])) / 1e3, 2),
                       "max_us": round(float(dur[:, i].max()) / 1e3, 2)}
                  for i, nm in enumerate(names) if nm != "-"}
        phases["page_start_us"] = {q: round(float(np.percentile(x[:, 0] - t0, q)) / 1e3, 1) for q in (0, 25, 50, 75, 100)}
        phases["page_end_us"] = {q: round(float(np.percentile(x[:, 10] - t0, q)) / 1e3, 1) for q in (0, 25, 50, 75, 100)}
        phases["page_life_p50_us"] = round(float(np.median(x[:, 10] - x[:, 0])) / 1e3, 1)
    print(json.dumps({"kernel": "k_seg_encode", "lib": a.lib or "built-in", "rows": n, "strings": not a.no_strings, "block_bytes": nb,
                      "bytes_per_row": round(nb / n, 3), "mean_us": round(float(np.mean(times)), 1),
                      "min_us": round(float(np.min(times)), 1), "reps": a.reps, "phases": phases}), flush=True)


if __name__ == "__main__":
    main()
