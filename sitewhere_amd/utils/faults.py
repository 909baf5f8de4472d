"""Seeded fault injection for resilience tests ("drop or delay bus deliveries",
transient storage / RPC failures).

``FaultInjector`` patches bound methods of live objects for the duration of a ``with`` block:

* ``fail(obj, "add_events", rate)``  -- the call raises :class:`InjectedFault` with probability ``rate``
  (before the real method runs, i.e. the side effect does not happen: a transient outage);
* ``fail_next(obj, "add_events", n)`` -- the next ``n`` calls raise (a deterministic outage);
* ``drop(obj, "read", rate, empty=[])`` -- the call returns ``empty`` instead (a lost / late delivery:
  for a log read the records come back on a later poll);
* ``delay(obj, "read", rate, seconds)`` -- the call sleeps first.

Decisions come from one seeded ``random.Random`` under a lock, so a failing run is reproducible in
the sequence of injected faults (thread interleavings aside).  Counters per (method, kind) are in
``injected``.
"""
from __future__ import annotations

import random
import threading
import time
from collections import Counter


class InjectedFault(RuntimeError):
    pass


class FaultInjector:
    def __init__(self, seed: int = 0):
        self._rng = random.Random(seed)
        self._lock = threading.Lock()
        self._patched: list[tuple[object, str, bool, object]] = []
        self.injected: Counter = Counter()
        self.enabled = True

    def _roll(self, rate: float) -> bool:
        if not self.enabled or rate <= 0:
            return False
        with self._lock:
            return self._rng.random() < rate

    def _patch(self, obj, name: str, make):
        had = name in getattr(obj, "__dict__", {})
        orig = getattr(obj, name)
        setattr(obj, name, make(orig))
        self._patched.append((obj, name, had, orig))

    def fail(self, obj, name: str, rate: float):
        def make(orig):
            def wrapped(*a, **kw):
                if self._roll(rate):
                    self.injected[(name, "fail")] += 1
                    raise InjectedFault(f"injected failure in {type(obj).__name__}.{name}")
                return orig(*a, **kw)
            return wrapped
        self._patch(obj, name, make)
        return self

    def fail_next(self, obj, name: str, n: int = 1):
        left = [n]

        def make(orig):
            def wrapped(*a, **kw):
                with self._lock:
                    hit = self.enabled and left[0] > 0
                    if hit:
                        left[0] -= 1
                if hit:
                    self.injected[(name, "fail")] += 1
                    raise InjectedFault(f"injected failure in {type(obj).__name__}.{name}")
                return orig(*a, **kw)
            return wrapped
        self._patch(obj, name, make)
        return self

    def drop(self, obj, name: str, rate: float, empty=None):
        def make(orig):
            def wrapped(*a, **kw):
                if self._roll(rate):
                    self.injected[(name, "drop")] += 1
                    return type(empty)() if isinstance(empty, (list, dict)) else empty
                return orig(*a, **kw)
            return wrapped
        self._patch(obj, name, make)
        return self

    def delay(self, obj, name: str, rate: float, seconds: float):
        def make(orig):
            def wrapped(*a, **kw):
                if self._roll(rate):
                    self.injected[(name, "delay")] += 1
                    time.sleep(seconds)
                return orig(*a, **kw)
            return wrapped
        self._patch(obj, name, make)
        return self

    def restore(self):
        self.enabled = False
        for obj, name, had, orig in reversed(self._patched):
            if had:
                setattr(obj, name, orig)
            else:
                try:
                    delattr(obj, name)
                except AttributeError:
                    pass
        self._patched.clear()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.restore()
        return False
