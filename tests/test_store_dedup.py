"""Store-backed alternate-id dedup beyond the engine's window.

An engine tenant (``gpu-columnar``: durable segment store, store-backed dedup filter on) stores a
device's payload, then forgets its whole dedup window (as after more than ``dedup_slots / 2`` newer
ids).  The device re-sends the payload: the window does not know it, the filter does, so the engine
hands it to the host (``SW_ST_RECHECK``), whose per-event path finds the id in the durable store and
reports a duplicate instead of storing it twice.  A new id sent at the same time is stored normally.

Reference: ``AlternateIdDeduplicator.java:41-56`` (asks event management for every event)."""
from __future__ import annotations

import os
import time

import pytest
from conftest import engine_knows

from sitewhere_amd.models import wire


def wait_until(cond, timeout=30.0, step=0.02):
    end = time.time() + timeout
    while time.time() < end:
        v = cond()
        if v:
            return v
        time.sleep(step)
    return cond()


@pytest.fixture
def sw(tmp_path):
    from sitewhere_amd.assembly import SiteWhereInstance
    old = os.environ.get("SITEWHERE_DATA_DIR")
    os.environ["SITEWHERE_DATA_DIR"] = str(tmp_path / "data")
    inst = SiteWhereInstance().start()
    inst.wait_for_tenant("default", 60)
    tm = inst.api("TenantManagement")
    inst.instance.system_user.run(lambda: tm.create_tenant({"token": "sd", "name": "sd",
                                                            "configurationTemplateId": "gpu-columnar",
                                                            "datasetTemplateId": "construction"}))
    inst.wait_for_tenant("sd", 60)
    yield inst
    inst.stop()
    if old is None:
        os.environ.pop("SITEWHERE_DATA_DIR", None)
    else:
        os.environ["SITEWHERE_DATA_DIR"] = old


def _measurements(sw, alt_prefix):
    run = lambda f: sw.instance.system_user.run(f, "sd")  # noqa: E731
    dm, em = sw.api("DeviceManagement", "sd"), sw.api("DeviceEventManagement", "sd")
    aid = run(lambda: dm.get_device_by_token("galaxytab-002")).device_assignment_id
    res = run(lambda: em.list_measurements_for_index("Assignment", [aid], {"pageSize": 0})).results
    return [m for m in res if (m.alternate_id or "").startswith(alt_prefix)]


def test_replay_beyond_the_window_is_a_duplicate(sw):
    ib = sw.tenant_engine("inbound-processing", "sd")
    assert ib.engine.cfg.dedup_filter_ids > 0
    es = sw.tenant_engine("event-sources", "sd")
    dev = sw.instance.system_user.run(lambda: sw.api("DeviceManagement", "sd").get_device_by_token("galaxytab-002"),
                                      "sd")
    assert wait_until(lambda: engine_knows(ib, dev), 30)
    first = wire.measurements("galaxytab-002", {"sd.temp": 1.5}, event_date=1_700_000_000_000, alternate_id="sd-old-1")
    es.inject("default-protobuf", first)
    assert wait_until(lambda: len(_measurements(sw, "sd-old-1")) == 1, 30)
    # the store's background index covers the stored block (the step's settle reads indexed
    # blocks only; an unindexed one leaves the id to the per-event path's own store check)
    store = sw.tenant_engine("event-management", "sd").store
    assert store.index_wait(30)
    # the window forgets everything (what more than dedup_slots / 2 newer ids would do)
    ib.engine.reset_dedup()
    s0 = ib.engine.stats_dict()
    es.inject("default-protobuf", first)                                             # the replay
    es.inject("default-protobuf", wire.measurements("galaxytab-002", {"sd.temp": 2.5}, event_date=1_700_000_001_000,
                                                    alternate_id="sd-new-1"))
    assert wait_until(lambda: len(_measurements(sw, "sd-new-1")) == 1, 30)
    assert wait_until(lambda: ib.engine.stats_dict()["dedup_rechecks"] > s0["dedup_rechecks"], 30)
    time.sleep(0.5)                                  # the host path has had time to store a second copy
    assert len(_measurements(sw, "sd-old-1")) == 1
    assert ib.engine.stats_dict()["duplicates"] == s0["duplicates"]        # the window did not see it
    # the store lookup found its hash (a replay); the per-event path compared the id strings and
    # dropped it (a hash match alone never drops an event)
    assert wait_until(lambda: ib.recheck_duplicates >= 1, 10)
    # a filter false positive (an id never stored whose fingerprint the filter holds) is stored by
    # the host path
    from sitewhere_amd.pipeline.fleet import hash64
    import numpy as np
    ib.engine.filter_seed_begin()
    ib.engine.filter_seed(np.array([hash64("sd-fp-1")], np.uint64))
    s1 = ib.engine.stats_dict()
    es.inject("default-protobuf", wire.measurements("galaxytab-002", {"sd.temp": 3.5}, event_date=1_700_000_002_000,
                                                    alternate_id="sd-fp-1"))
    assert wait_until(lambda: len(_measurements(sw, "sd-fp-1")) == 1, 30)
    assert ib.engine.stats_dict()["dedup_rechecks"] == s1["dedup_rechecks"] + 1
    assert _measurements(sw, "sd-fp-1")[0].value == 3.5
