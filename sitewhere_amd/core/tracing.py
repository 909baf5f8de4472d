"""Distributed tracing (OpenTracing-style) with probabilistic sampling.

Reference: the Jaeger tracer bean (``MicroserviceConfiguration.java:51-58``, sampler 0.01),
``TracerUtils.java:25-60`` (error tagging) and the gRPC ``ServerTracingInterceptor`` /
``ClientTracingInterceptor`` that the reference never switches on.  Here tracing is on by
default on the hot path: spans propagate through :mod:`contextvars` and across RPC and bus
hops as a ``uber-trace-id``-style header (``trace_id:span_id:parent_id:flags``).
"""
from __future__ import annotations

import contextvars
import random
import threading
import time
from collections import deque
from dataclasses import dataclass, field
from ..utils import fast_hex

_current: contextvars.ContextVar["Span | None"] = contextvars.ContextVar("sw_span", default=None)
HEADER = "uber-trace-id"


@dataclass
class Span:
    tracer: "Tracer"
    name: str
    trace_id: str
    span_id: str
    parent_id: str | None
    sampled: bool
    start: float = field(default_factory=time.time)
    end: float | None = None
    tags: dict = field(default_factory=dict)
    logs: list = field(default_factory=list)
    _token: object = None

    def set_tag(self, k, v):
        self.tags[k] = v
        return self

    def log(self, **fields):
        self.logs.append({"ts": time.time(), **fields})
        return self

    def set_error(self, exc: BaseException):
        """TracerUtils.handleErrorInTracerSpan equivalent."""
        self.tags["error"] = True
        self.logs.append({"ts": time.time(), "event": "error", "error.kind": type(exc).__name__,
                          "message": str(exc)})
        return self

    def finish(self):
        if self.end is None:
            self.end = time.time()
            self.tracer._report(self)

    def context_header(self) -> str:
        return f"{self.trace_id}:{self.span_id}:{self.parent_id or 0}:{1 if self.sampled else 0}"

    def __enter__(self):
        self._token = _current.set(self)
        return self

    def __exit__(self, et, ev, tb):
        if ev is not None:
            self.set_error(ev)
        self.finish()
        if self._token is not None:
            _current.reset(self._token)
        return False

    @property
    def duration_ms(self):
        return None if self.end is None else (self.end - self.start) * 1000


class Tracer:
    """Tracer with a probabilistic sampler and an in-memory ring reporter."""

    def __init__(self, service: str = "sitewhere", sample_rate: float = 0.01, capacity: int = 10000,
                 reporter=None):
        self.service = service
        self.sample_rate = sample_rate
        self.finished: deque = deque(maxlen=capacity)
        self.reporter = reporter
        self._lock = threading.Lock()

    def start_span(self, name: str, child_of: Span | str | None = None, force_sample: bool = False) -> Span:
        parent = child_of if child_of is not None else _current.get()
        if isinstance(parent, str):
            parent = self.extract(parent)
        if parent is not None:
            trace_id, parent_id, sampled = parent.trace_id, parent.span_id, parent.sampled
        else:
            trace_id, parent_id = fast_hex(64), None
            sampled = force_sample or random.random() < self.sample_rate
        return Span(self, name, trace_id, fast_hex(64), parent_id, sampled,
                    tags={"service": self.service})

    def extract(self, header: str | None) -> Span | None:
        if not header:
            return None
        try:
            t, s, p, f = header.split(":")
        except ValueError:
            return None
        return Span(self, "remote", t, s, None if p == "0" else p, f == "1")

    @staticmethod
    def active() -> Span | None:
        return _current.get()

    def _report(self, span: Span):
        if not span.sampled:
            return
        with self._lock:
            self.finished.append(span)
        if self.reporter:
            try:
                self.reporter(span)
            except Exception:
                pass

    def export(self) -> list[dict]:
        with self._lock:
            spans = list(self.finished)
        return [{"name": s.name, "traceId": s.trace_id, "spanId": s.span_id, "parentId": s.parent_id,
                 "start": s.start, "durationMs": s.duration_ms, "tags": s.tags, "logs": s.logs} for s in spans]


_global = Tracer()


def global_tracer() -> Tracer:
    return _global


def set_global_tracer(t: Tracer):
    global _global
    _global = t
