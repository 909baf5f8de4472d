"""Runtime dedup sizing check: an engine tenant warns when its HBM dedup window is
smaller than what the raw topic can redeliver and no store-backed filter is configured, when its
durable store may keep more rows than the generational filter holds ids (retention by
rows must bound the store), and when in-flight false positives pass 1e-4 of the payloads."""
from __future__ import annotations

import logging
from types import SimpleNamespace

from sitewhere_amd.pipeline.config import EngineConfig
from sitewhere_amd.services.gpu_inbound import GpuInboundTenantEngine as T


class _Bus:
    def __init__(self, retention, parts=4):
        self._r, self._p = retention, parts

    def retention(self, name):
        return self._r

    def partitions(self, name):
        return self._p


def _tenant(cfg, retention, stored=0, limit=0):
    return SimpleNamespace(engine_cfg=cfg, ms=SimpleNamespace(instance=SimpleNamespace(bus=_Bus(retention))),
                           raw_consumer=SimpleNamespace(topics=["t1.raw"]), logger=logging.getLogger("sizing"),
                           MIN_PAYLOAD_BYTES=T.MIN_PAYLOAD_BYTES, storage="durable", filter_retention_rows=limit,
                           engine=SimpleNamespace(filter_state=lambda: {}),
                           _stored_ids=stored, dedup_sizing_report={}, _fp_win=[0, 0])


def test_window_smaller_than_redelivery_warns_without_filter(caplog):
    cfg = EngineConfig.small(dedup_slots=1 << 16)
    with caplog.at_level(logging.WARNING, "sizing"):
        rep = T.check_dedup_sizing(_tenant(cfg, retention=1 << 30))
    assert rep["raw_redeliverable_ids"] == 4 * ((1 << 30) // T.MIN_PAYLOAD_BYTES)
    assert len(rep["warnings"]) == 1 and "dedup_slots" in rep["warnings"][0]
    assert any("dedup window" in r.message for r in caplog.records)
    # unlimited retention: still a warning
    assert T.check_dedup_sizing(_tenant(cfg, retention=0))["raw_redeliverable_ids"] is None
    # a window larger than the topic can hold: fine
    small = T.check_dedup_sizing(_tenant(EngineConfig.small(dedup_slots=1 << 20), retention=1 << 16))
    assert small["warnings"] == []


def test_store_rows_bounded_by_what_the_filter_holds():
    cfg = EngineConfig.small(dedup_slots=1 << 16, dedup_filter_ids=1 << 20, dedup_filter_gens=4)
    held = 3 * (1 << 20)
    assert cfg.filter_retention_rows(0) == int(held / 1.25)               # the file being written
    assert cfg.filter_retention_rows(1 << 20) == int((held - (1 << 20)) / 1.25)
    rep = T.check_dedup_sizing(_tenant(cfg, retention=0, limit=cfg.filter_retention_rows(1 << 20)))
    assert rep["warnings"] == [] and rep["filter_holds_ids"] == held
    # the store's row limit could not be set (or is above what the filter holds): replays of older
    # stored ids would pass
    rep = T.check_dedup_sizing(_tenant(cfg, retention=0, limit=0))
    assert len(rep["warnings"]) == 1 and "not caught" in rep["warnings"][0]
    rep = T.check_dedup_sizing(_tenant(cfg, retention=0, limit=held + 1))
    assert len(rep["warnings"]) == 1


def test_false_positive_watch(caplog):
    t = _tenant(EngineConfig.small(dedup_filter_ids=1 << 16), retention=0)
    with caplog.at_level(logging.WARNING, "sizing"):
        T._watch_filter(t, 1 << 21, 100)
        T._watch_filter(t, 1 << 21, 100)           # 0.005%: quiet
        assert not caplog.records and t._fp_win == [0, 0]
        T._watch_filter(t, 1 << 22, 1 << 16)       # 1.6%: a mis-sized filter
    assert any("false positives" in r.message for r in caplog.records)
