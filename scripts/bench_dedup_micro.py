"""Driver of scripts/dedup_micro.hip: times each claim mode on synthetic ids (1.3M records of 80 B, an
id each; the retired generation is 40% full of other ids; the live one starts empty each rep), HIP events.
Prints one JSON line per (mode, grid).

    python scripts/bench_dedup_micro.py [--n 1310720] [--slots 4194304]"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

MODES = {0: "engine claim", 1: "CAS only", 2: "prev probe only", 3: "probe || CAS", 4: "2 ids in flight",
         5: "id + status loads"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1310720)
    ap.add_argument("--slots", type=int, default=1 << 22)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--lib", default="sitewhere_amd/_lib/variants/libdedup_micro.so")
    a = ap.parse_args()
    import torch
    from ctypes import c_int, c_int32, c_int64, c_void_p as P
    from sitewhere_amd.models.columnar import EVENT_REC
    lib = ctypes.CDLL(os.path.abspath(a.lib))
    lib.dm_claim.restype = c_int32
    lib.dm_claim.argtypes = [P, P, c_int64, P, P, c_int64, c_int, c_int, P, P]
    d = torch.device("cuda", 0)
    rng = np.random.default_rng(5)
    recs = np.zeros(a.n, EVENT_REC)
    recs["alt_hash"] = rng.integers(2, 1 << 62, a.n, dtype=np.int64).astype(np.uint64)
    recs_t = torch.from_numpy(recs.view(np.uint8)).to(d)
    # retired generation: 40% full of other ids, linear probing (host-built)
    mask = a.slots - 1
    prev = np.zeros(2 * a.slots, np.uint64)
    for h in rng.integers(2, 1 << 62, a.slots * 2 // 5, dtype=np.int64).astype(np.uint64).tolist():
        s = h & mask
        while prev[2 * s]:
            s = (s + 1) & mask
        prev[2 * s] = h
    prev_t = torch.from_numpy(prev.view(np.int64)).to(d)
    cur_t = torch.zeros(2 * a.slots, dtype=torch.int64, device=d)
    status_t = torch.zeros(a.n, dtype=torch.uint8, device=d)
    sink = torch.zeros(1, dtype=torch.int64, device=d)
    s = torch.cuda.current_stream(d)
    for mode in MODES:
        for grid in (2048, 4096, 8192):
            ts = []
            for r in range(a.reps + 2):
                cur_t.zero_()
                status_t.zero_()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                assert lib.dm_claim(P(recs_t.data_ptr()), P(status_t.data_ptr()), a.n, P(cur_t.data_ptr()),
                                    P(prev_t.data_ptr()), mask, mode, grid, P(sink.data_ptr()), P(s.cuda_stream)) == 0
                e1.record(s)
                s.synchronize()
                if r >= 2:
                    ts.append(1000.0 * e0.elapsed_time(e1))
            print(json.dumps({"mode": mode, "what": MODES[mode], "grid": grid, "ids": a.n, "slots": a.slots,
                              "mean_us": round(float(np.mean(ts)), 1), "min_us": round(float(np.min(ts)), 1)}),
                  flush=True)
    del prev_t, cur_t
    updates(lib, recs_t, a.n, d, a.reps)


def updates(lib, recs_t, n, d, reps):
    """Scattered persist-side updates (modes 6-9 of dedup_micro.hip) into an 8 GiB word table."""
    import torch
    from ctypes import c_int, c_int32, c_int64, c_void_p as P
    lib.dm_update.restype = c_int32
    lib.dm_update.argtypes = [P, c_int64, P, c_int64, c_int, c_int, P]
    words = 1 << 30
    tab = torch.zeros(words, dtype=torch.int64, device=d)
    s = torch.cuda.current_stream(d)
    what = {6: "atomicOr no-return (filter add)", 7: "plain load+store", 8: "atomicMax 32B slots",
            9: "checked plain store 32B slots"}
    for mode, w in what.items():
        for grid in (2048, 8192):
            ts = []
            for r in range(reps + 2):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                assert lib.dm_update(P(recs_t.data_ptr()), n, P(tab.data_ptr()), words - 1, mode, grid,
                                     P(s.cuda_stream)) == 0
                e1.record(s)
                s.synchronize()
                if r >= 2:
                    ts.append(1000.0 * e0.elapsed_time(e1))
            print(json.dumps({"mode": mode, "what": w, "grid": grid, "ids": n, "table_words": words,
                              "mean_us": round(float(np.mean(ts)), 1), "min_us": round(float(np.min(ts)), 1)}),
                  flush=True)
    del tab


if __name__ == "__main__":
    main()
