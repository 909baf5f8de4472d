"""Read load on a durable event store while it ingests: the REST / gRPC query mix of the reference's
event-management API (ListMeasurementsForIndex on Assignment, Area, Customer and Asset,
GetDeviceEventById, GetDeviceEventByAlternateId) issued from reader threads against the store the
engine is writing, each query timed.

Reference: service-event-management DeviceEventManagementImpl (listDeviceMeasurementsForIndex,
getDeviceEventById, getDeviceEventByAlternateId) over MongoDeviceEventManagement.java:129-141's
indexes -- here answered from the block index trailers built on the GPU in the ingest step.

Used by ``bench.py --read-threads N`` (latencies in the bench line's ``detail.reads``) and by
``scripts/bench_store_reads.py``."""
from __future__ import annotations

import threading
import time

import numpy as np

from ..models.domain import DateRangeSearchCriteria

KINDS = ("list_assignment", "list_area", "list_customer", "list_asset", "by_id", "by_alt", "by_alt_miss")
_LIST = {"list_assignment": ("Assignment", "asg", "n_asg"), "list_area": ("Area", "area", "n_area"),
         "list_customer": ("Customer", "cust", "n_cust"), "list_asset": ("Asset", "asset", "n_asset")}


def bench_dictionary(n_assignments: int, n_cust: int = 97, n_area: int = 31, n_asset: int = 1009):
    """The dictionary of bench.py's fleet (assignment i -> device i, customer i % n_cust, area
    i % n_area, asset i % n_asset; n_asset 0: one asset per device) and the engine's context ids of
    those tokens."""
    n_asset = n_asset or n_assignments
    asg = {i: [f"asg-{i}", f"dev-{i}", f"cust-{i % n_cust}", f"area-{i % n_area}", f"asset-{i % n_asset}"]
           for i in range(n_assignments)}
    ctx = {0: {f"cust-{k}": k for k in range(n_cust)}, 1: {f"area-{k}": k for k in range(n_area)},
           2: {f"asset-{k}": k for k in range(n_asset)}}
    return asg, ctx


class ReadLoad:
    """``threads`` readers cycling through :data:`KINDS` against ``store`` until :meth:`stop`.

    Targets: assignments ``asg-<i>`` (i < ``n_assignments``), areas ``area-<k>`` (k < ``n_area``),
    customers ``cust-<k>`` (k < ``n_cust``), assets ``asset-<k>`` (k < ``n_asset``), and stored events picked at random from the blocks already durable (their ids, then the
    alternate ids those events carry).  ``pause_s`` between queries per thread (0: back to back)."""

    def __init__(self, store, n_assignments: int, n_area: int = 31, threads: int = 2, pause_s: float = 0.0,
                 page_size: int = 100, seed: int = 7, n_cust: int = 97, n_asset: int = 1009):
        self.store = store
        self.n_asg, self.n_area = int(n_assignments), int(n_area)
        self.n_cust, self.n_asset = int(n_cust), int(n_asset or n_assignments)
        self.threads, self.pause_s, self.page_size = int(threads), float(pause_s), int(page_size)
        self.seed = seed
        self.lat = {k: [] for k in KINDS}
        self.phases = {k: [] for k in KINDS if k.startswith("list")}   # per query: {phase: seconds}
        self.results = {k: [] for k in KINDS}
        self.errors: list[str] = []
        self._stop = threading.Event()
        self._th: list[threading.Thread] = []

    def _pick_event_id(self, rng) -> str | None:
        ents = self.store.seg.index()
        ents = ents[ents["n_rows"] > 0]
        if not len(ents):
            return None
        e = ents[int(rng.integers(0, len(ents)))]
        row = int(rng.integers(0, int(e["n_rows"])))
        eid = (int(e["first_seq"]) + row) * int(e["world"]) + int(e["rank"])
        return f"{int(e['boot']):x}-{eid}"

    def _one(self, kind: str, rng):
        st = self.store
        crit = DateRangeSearchCriteria(page_size=self.page_size)
        if kind in _LIST:
            ix, prefix, n = _LIST[kind]
            ent = f"{prefix}-{int(rng.integers(0, getattr(self, n)))}"
            t = time.perf_counter()
            r = st.list_events("Measurement", ix, [ent], crit)
            dt = time.perf_counter() - t
            tl = getattr(st, "_tl", None)
            if tl is not None and getattr(tl, "phases", None) is not None:
                self.phases[kind].append(dict(tl.phases, total=dt))
            return dt, r.num_results
        if kind == "by_alt_miss":
            t = time.perf_counter()
            ev = st.get_event_by_alternate_id(f"never-stored-{int(rng.integers(0, 1 << 40))}")
            dt = time.perf_counter() - t
            if ev is not None:
                self.errors.append("a never-stored alternate id was found")
            return dt, 0
        id_ = self._pick_event_id(rng)
        if id_ is None:
            return None
        t = time.perf_counter()
        ev = st.get_event_by_id(id_)
        dt = time.perf_counter() - t
        if ev is None or ev.id != id_:
            self.errors.append(f"event {id_} not found by id")
            return dt, 0
        if kind == "by_id":
            return dt, 1
        if not ev.alternate_id:
            return None
        t = time.perf_counter()
        ev2 = st.get_event_by_alternate_id(ev.alternate_id)
        dt = time.perf_counter() - t
        if ev2 is None or ev2.alternate_id != ev.alternate_id:
            self.errors.append(f"alternate id {ev.alternate_id} not found")
        return dt, 1

    def _run(self, k: int):
        rng = np.random.default_rng(self.seed + k)
        i = k
        while not self._stop.is_set():
            kind = KINDS[i % len(KINDS)]
            i += 1
            try:
                got = self._one(kind, rng)
            except Exception as e:        # noqa: BLE001 -- a failing query is reported, not fatal to ingest
                self.errors.append(f"{kind}: {type(e).__name__}: {e}")
                got = None
            if got is not None:
                self.lat[kind].append(got[0])
                self.results[kind].append(got[1])
            if self.pause_s:
                self._stop.wait(self.pause_s)

    def start(self):
        self._stop.clear()
        self._th = [threading.Thread(target=self._run, args=(k,), name=f"read-load-{k}", daemon=True)
                    for k in range(self.threads)]
        for t in self._th:
            t.start()
        return self

    def stop(self) -> dict:
        self._stop.set()
        for t in self._th:
            t.join()
        return self.summary()

    def summary(self) -> dict:
        out = {"threads": self.threads, "page_size": self.page_size, "errors": self.errors[:5],
               "n_errors": len(self.errors)}
        for k in KINDS:
            v = np.asarray(self.lat[k]) * 1e3
            if len(v):
                out[k + "_ms"] = {"n": int(len(v)), "p50": round(float(np.percentile(v, 50)), 3),
                                  "p99": round(float(np.percentile(v, 99)), 3), "max": round(float(v.max()), 3)}
                if k.startswith("list"):
                    out[k + "_ms"]["results_mean"] = round(float(np.mean(self.results[k])), 1)
                    ph = self.phases.get(k) or []
                    if ph:
                        # the phases of the slowest 5% of the queries, and the median query's
                        tot = np.array([p["total"] for p in ph])
                        slow = [ph[i] for i in np.argsort(tot)[-max(1, len(ph) // 20):]]
                        mid = ph[int(np.argsort(tot)[len(ph) // 2])]
                        keys = sorted({x for p in ph for x in p if x != "total"})
                        sc = {x: 1.0 if x.endswith("_n") else 1e3 for x in keys + ["total"]}   # "_n": counts
                        out[k + "_ms"]["phases_p50_query"] = {x: round(sc[x] * mid.get(x, 0.0), 3) for x in keys}
                        out[k + "_ms"]["phases_slowest5pct_mean"] = {
                            x: round(sc[x] * float(np.mean([p.get(x, 0.0) for p in slow])), 3) for x in keys + ["total"]}
        return out
