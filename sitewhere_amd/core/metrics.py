"""Metrics registry (Dropwizard-equivalent) with Prometheus text exposition.

Reference: per-process ``MetricRegistry``; meters/timers named ``<tenantPrefix><name>``
(``TenantEngineLifecycleComponent.java:45-56``) and reported every 20 s when
``sitewhere.log.metrics`` is set (``Microservice.java:242-250``).  The reference has no
exporter; :meth:`MetricRegistry.prometheus` provides one.
"""
from __future__ import annotations

import math
import re
import itertools
import threading
import time
from collections import deque


class Counter:
    def __init__(self):
        self._v = 0
        self._lock = threading.Lock()

    def inc(self, n: int = 1):
        with self._lock:
            self._v += n

    def dec(self, n: int = 1):
        self.inc(-n)

    @property
    def count(self):
        return self._v


class Meter:
    """Count plus exponentially-weighted 1/5/15-minute rates."""

    def __init__(self):
        self._count = 0
        self._start = time.time()
        self._last_tick = self._start
        self._rates = [0.0, 0.0, 0.0]
        self._uncounted = 0
        self._lock = threading.Lock()

    _ALPHA = [1 - math.exp(-5 / 60.0), 1 - math.exp(-5 / 300.0), 1 - math.exp(-5 / 900.0)]

    def _tick_if_needed(self):
        now = time.time()
        while now - self._last_tick >= 5.0:
            inst = self._uncounted / 5.0
            self._uncounted = 0
            for i, a in enumerate(self._ALPHA):
                self._rates[i] += a * (inst - self._rates[i])
            self._last_tick += 5.0

    def mark(self, n: int = 1):
        # no lock on the hot path: += on ints is effectively atomic for these counters under the GIL
        # (a lost update can only skew a rate estimate); ticking takes the lock
        self._count += n
        self._uncounted += n
        if time.time() - self._last_tick >= 5.0:
            with self._lock:
                self._tick_if_needed()

    @property
    def count(self):
        return self._count

    def mean_rate(self):
        el = time.time() - self._start
        return self._count / el if el > 0 else 0.0

    def rates(self):
        with self._lock:
            self._tick_if_needed()
            return tuple(self._rates)


class Histogram:
    """Sliding reservoir of the last ``reservoir`` values.  Lock-free on the update path: a bounded
    ``deque.append`` and ``next(itertools.count)`` are atomic under the GIL, whereas a lock taken by
    every processing thread convoys behind the GIL switch interval (measured: ~1 ms per update)."""

    def __init__(self, reservoir: int = 1028):
        self._vals: deque = deque(maxlen=reservoir)
        self._counter = itertools.count(1)
        self._count = 0

    def update(self, v: float):
        self._vals.append(v)
        self._count = next(self._counter)

    @property
    def count(self):
        return self._count

    def snapshot(self):
        vals = sorted(list(self._vals))
        if not vals:
            return {"count": self._count, "min": 0, "max": 0, "mean": 0, "p50": 0, "p95": 0, "p99": 0}

        def q(p):
            return vals[min(len(vals) - 1, int(p * len(vals)))]

        return {"count": self._count, "min": vals[0], "max": vals[-1], "mean": sum(vals) / len(vals),
                "p50": q(0.5), "p95": q(0.95), "p99": q(0.99)}


class Timer:
    """Meter + histogram of durations in milliseconds.  Use as a context manager."""

    def __init__(self):
        self.meter = Meter()
        self.hist = Histogram()

    def update(self, ms: float):
        self.meter.mark()
        self.hist.update(ms)

    def time(self):
        return _TimerCtx(self)

    @property
    def count(self):
        return self.meter.count


class _TimerCtx:
    def __init__(self, t: Timer):
        self.t = t

    def __enter__(self):
        self.s = time.perf_counter()
        return self

    def __exit__(self, *a):
        self.t.update((time.perf_counter() - self.s) * 1000)
        return False


class Gauge:
    def __init__(self, fn):
        self.fn = fn

    @property
    def value(self):
        try:
            return self.fn()
        except Exception:
            return float("nan")


class MetricRegistry:
    def __init__(self):
        self._m: dict = {}
        self._lock = threading.Lock()

    def _get(self, name, cls, *a):
        with self._lock:
            m = self._m.get(name)
            if m is None:
                m = cls(*a)
                self._m[name] = m
            elif not isinstance(m, cls):
                raise TypeError(f"metric {name} already registered as {type(m).__name__}")
            return m

    def counter(self, name) -> Counter:
        return self._get(name, Counter)

    def meter(self, name) -> Meter:
        return self._get(name, Meter)

    def timer(self, name) -> Timer:
        return self._get(name, Timer)

    def histogram(self, name) -> Histogram:
        return self._get(name, Histogram)

    def gauge(self, name, fn) -> Gauge:
        return self._get(name, Gauge, fn)

    def names(self):
        with self._lock:
            return sorted(self._m)

    def get(self, name):
        return self._m.get(name)

    def snapshot(self) -> dict:
        out = {}
        with self._lock:
            items = list(self._m.items())
        for n, m in items:
            if isinstance(m, Counter):
                out[n] = {"type": "counter", "count": m.count}
            elif isinstance(m, Meter):
                r = m.rates()
                out[n] = {"type": "meter", "count": m.count, "mean_rate": m.mean_rate(), "m1": r[0], "m5": r[1],
                          "m15": r[2]}
            elif isinstance(m, Timer):
                out[n] = {"type": "timer", **m.hist.snapshot(), "mean_rate": m.meter.mean_rate()}
            elif isinstance(m, Histogram):
                out[n] = {"type": "histogram", **m.snapshot()}
            elif isinstance(m, Gauge):
                out[n] = {"type": "gauge", "value": m.value}
        return out

    def prometheus(self, prefix: str = "sitewhere_") -> str:
        lines = []
        for n, v in self.snapshot().items():
            pn = prefix + re.sub(r"[^a-zA-Z0-9_]", "_", n)
            t = v["type"]
            if t in ("counter", "meter"):
                lines += [f"# TYPE {pn}_total counter", f"{pn}_total {v['count']}"]
            elif t in ("timer", "histogram"):
                lines += [f"# TYPE {pn}_ms summary"]
                for q in ("p50", "p95", "p99"):
                    lines.append(f'{pn}_ms{{quantile="0.{q[1:]}"}} {v[q]}')
                lines.append(f"{pn}_ms_count {v['count']}")
            elif t == "gauge":
                lines += [f"# TYPE {pn} gauge", f"{pn} {v['value']}"]
        return "\n".join(lines) + "\n"


class MetricsReporter(threading.Thread):
    """Periodic reporter (reference Slf4jReporter every 20 s)."""

    def __init__(self, registry: MetricRegistry, sink, period_s: float = 20.0):
        super().__init__(daemon=True, name="metrics-reporter")
        self.registry, self.sink, self.period = registry, sink, period_s
        self._stop = threading.Event()

    def run(self):
        while not self._stop.wait(self.period):
            try:
                self.sink(self.registry.snapshot())
            except Exception:
                pass

    def stop(self):
        self._stop.set()
