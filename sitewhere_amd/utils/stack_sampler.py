"""Wall-clock stack sampler for a service process (``SW_STACK_SAMPLE=<path prefix>``).

A daemon thread snapshots every thread's Python stack (``sys._current_frames``) every
``SW_STACK_SAMPLE_MS`` (default 5) and counts, per thread name, the innermost frame and every
function on the stack (inclusive).  Threads parked in a wait (queue get, lock / event wait, sleep,
select, socket receive) are counted apart, so the busy profile shows where CPU and GIL time goes.
At exit the counts are written to ``<prefix>.<pid>.txt``.  What the reference gets from a JVM
profiler attached to a pod; here it finds the hot path of a per-event service (profiles/r6_per_event)."""
from __future__ import annotations

import atexit
import collections
import os
import sys
import threading
import time
import traceback

_IDLE = {"wait", "get", "sleep", "select", "poll", "recv", "recv_into", "accept", "_wait_for_tstate_lock",
         "acquire", "readinto", "_recv", "read_packet", "_worker", "wait_for"}


class StackSampler:
    def __init__(self, path: str, interval_s: float = 0.005):
        self.path, self.interval = path, interval_s
        self.leaf = collections.defaultdict(collections.Counter)
        self.incl = collections.defaultdict(collections.Counter)
        self.idle = collections.Counter()
        self.busy = collections.Counter()
        self.rounds = 0
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, name="stack-sampler", daemon=True)

    def start(self):
        self._t.start()
        atexit.register(self.dump)
        return self

    def _run(self):
        me = threading.get_ident()
        while not self._stop.wait(self.interval):
            names = {t.ident: t.name for t in threading.enumerate()}
            self.rounds += 1
            for tid, fr in sys._current_frames().items():
                if tid == me:
                    continue
                st = traceback.extract_stack(fr)
                if not st:
                    continue
                name = names.get(tid, str(tid)).rstrip("0123456789_-")
                if st[-1].name in _IDLE:
                    self.idle[name] += 1
                    continue
                self.busy[name] += 1
                self.leaf[name][f"{os.path.basename(st[-1].filename)}:{st[-1].lineno}:{st[-1].name}"] += 1
                seen = set()
                for f in st:
                    k = f"{os.path.basename(f.filename)}:{f.name}"
                    if k not in seen:
                        seen.add(k)
                        self.incl[name][k] += 1

    def dump(self):
        self._stop.set()
        try:
            with open(f"{self.path}.{os.getpid()}.txt", "w") as f:
                f.write(f"samples: {self.rounds} rounds of {self.interval * 1000:.1f} ms\n")
                for name, n in self.busy.most_common():
                    f.write(f"\n== thread {name}: busy {n}, idle {self.idle.get(name, 0)}\n-- innermost\n")
                    for k, v in self.leaf[name].most_common(25):
                        f.write(f"{v:7d} {k}\n")
                    f.write("-- inclusive\n")
                    for k, v in self.incl[name].most_common(40):
                        f.write(f"{v:7d} {k}\n")
        except OSError:
            pass


def maybe_start() -> StackSampler | None:
    p = os.environ.get("SW_STACK_SAMPLE")
    if not p:
        return None
    return StackSampler(p, float(os.environ.get("SW_STACK_SAMPLE_MS", "5")) / 1000.0).start()
