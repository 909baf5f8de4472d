"""Engine tenants keep every event they acknowledge, on every path (VERDICT r3 missing #3, #4).

* REST-added events (a measurement, a command invocation, its response) on a ``gpu-columnar`` tenant
  are on disk when the call returns: a process killed right after (``os._exit``) leaves them in the
  durable store, which a fresh :class:`DurableEventStore` over the same directory serves by id,
  alternate id and invocation.
* JSON device requests are transcoded onto the engine path (``csrc/native/swjson.cpp``) and stored
  whole: alert message, alternate id and metadata read back over REST, and again from the files
  after the kill.

Reference: ``DeviceEventBuffer.java:99-135`` (buffered Mongo writes, lost on a crash: SURVEY §5.4),
``JsonDeviceRequestDecoder.java``, ``DeviceEventManagementImpl`` adds."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def test_rest_adds_and_json_events_survive_a_kill(tmp_path):
    data = str(tmp_path / "data")
    p = subprocess.run([sys.executable, os.path.join(HERE, "api_durable_child.py")], capture_output=True, text=True,
                       timeout=300, env=dict(os.environ, SITEWHERE_DATA_DIR=data))
    assert p.returncode == 9, p.stderr[-3000:]
    out = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")][-1]
    # ---- JSON events through the engine, read back over REST before the kill
    js = out["json"]
    assert set(js) == {"json-a-1", "json-m-1", "json-l-1"}, js
    a = js["json-a-1"]
    assert (a["type"], a["message"], a["source"], a["level"]) == ("door.open", "door opened at gate 3", "Device", "Info")
    assert a["metadata"] == {"gate": "3", "shift": "night"} and a["alternateId"] == "json-a-1"
    assert js["json-m-1"]["name"] == "json.temp" and js["json-m-1"]["value"] == 21.25
    assert js["json-m-1"]["metadata"] == {"unit": "C"}
    assert js["json-l-1"]["elevation"] == 301.5

    # ---- after the kill: a fresh store over the files serves everything
    from sitewhere_amd.models.domain import DeviceEventType
    from sitewhere_amd.persistence.segments import DurableEventStore
    st = DurableEventStore(os.path.join(data, "dur", "events"))
    try:
        m = st.get_event_by_alternate_id("api-m-1")
        assert m is not None and m.id == out["measurement"]["id"] and m.value == 12.5 and m.metadata == {"src": "rest"}
        inv = st.get_event_by_id(out["invocation"]["id"])
        assert inv is not None and inv.event_type == DeviceEventType.CommandInvocation
        assert inv.parameter_values == {"message": "hi"}
        rs = st.list_command_responses_for_invocation(out["invocation"]["id"]).results
        assert [r.id for r in rs] == [out["response"]["id"]] and rs[0].response == "done"
        assert st.get_event_by_alternate_id("api-r-1").id == out["response"]["id"]
        for alt, want in js.items():
            assert st._objects.get_event_by_alternate_id(alt) is None     # a row of an engine block
            ev = st.get_event_by_alternate_id(alt)
            assert ev is not None and ev.id == want["id"], alt
            d = ev.to_dict()
            for k in ("message", "metadata", "alternateId", "value", "name", "elevation", "type"):
                if k in want:
                    assert d.get(k) == want[k], (alt, k)
    finally:
        st.close()


def _crash(st):
    """Stop a store the way a kill would: no tail flush, no close of the API log."""
    st._api_stop.set()
    st._api_kick.set()
    st._api_th.join()
    st.seg.close()


def test_api_log_torn_tail_is_cut(tmp_path, monkeypatch):
    """A crash mid-append leaves a partial line: reopening drops it and keeps every whole event."""
    monkeypatch.setenv("SW_API_FLUSH_S", "3600")         # nothing leaves the tail on its own
    from sitewhere_amd.models.domain import DeviceMeasurement
    from sitewhere_amd.persistence.segments import DurableEventStore
    d = str(tmp_path / "s")
    st = DurableEventStore(d, direct=False)
    evs = [DeviceMeasurement(name="t", value=float(i), event_date=1000 + i, device_assignment_id="a1",
                             alternate_id=f"alt-{i}") for i in range(5)]
    st.add_events(evs[:3])
    st.add_events(evs[3:])
    ids = [e.id for e in evs]
    assert len(set(ids)) == 5 and all(i.split("-")[0] == f"{st._api_boot:x}" for i in ids)
    _crash(st)
    path = os.path.join(d, "api-0.log")
    size = os.path.getsize(path)
    with open(path, "r+b") as f:
        f.truncate(size - 7)                  # tear the last event's line
    st = DurableEventStore(d, direct=False)
    try:
        assert [st.get_event_by_id(i) is not None for i in ids] == [True] * 4 + [False]
        assert os.path.getsize(path) < size - 7              # the torn line itself was cut off
        again = DeviceMeasurement(name="t", value=4.0, event_date=1004, device_assignment_id="a1", alternate_id="alt-4")
        st.add_events([again])
        assert again.id not in ids[:4]                        # sequences continue past the log's
    finally:
        st.close()
    st = DurableEventStore(d, direct=False)
    try:
        assert st.get_event_by_alternate_id("alt-4").value == 4.0 and st.count() == 5
        assert len(st._api_tail) == 0                         # close flushed the tail into a block
    finally:
        st.close()


def _api_events(n, seed=0):
    from sitewhere_amd.models.domain import (AlertLevel, AlertSource, DeviceAlert, DeviceCommandInvocation,
                                             DeviceCommandResponse, DeviceLocation, DeviceMeasurement,
                                             DeviceStateChange)
    out = []
    for i in range(seed, seed + n):
        ctx = dict(device_assignment_id=f"asg-{i % 7}", device_id=f"dev-{i % 7}", customer_id=f"cust-{i % 3}",
                   area_id=f"area-{i % 2}", asset_id=None if i % 5 == 0 else f"asset-{i % 4}", event_date=1_000_000 + i,
                   received_date=2_000_000 + i)
        k = i % 7
        if k == 0:
            e = DeviceMeasurement(name=f"m{i % 3}", value=i * 0.5, alternate_id=f"api-{i}", metadata={"u": "C"}, **ctx)
        elif k == 1:
            e = DeviceLocation(latitude=33.0 + i * 1e-4, longitude=-84.0, elevation=None if i % 2 else 12.5, **ctx)
        elif k == 2:
            e = DeviceAlert(source=AlertSource.Device, level=AlertLevel.Warning, type="door", message=f"open {i}",
                            metadata={"g": str(i)}, **ctx)
        elif k == 3:
            e = DeviceAlert(source=AlertSource.System, level=AlertLevel.Critical, type="rule.hot", message=f"hot {i}",
                            **ctx)
        elif k == 4:
            e = DeviceCommandInvocation(command_token="reboot", parameter_values={"delay": str(i)},
                                        target_id=ctx["device_assignment_id"], initiator_id="admin",
                                        alternate_id=f"inv-{i}", **ctx)
        elif k == 5:
            e = DeviceCommandResponse(originating_event_id=f"orig-{i}", response="ok", metadata={"r": "1"}, **ctx)
        else:
            e = DeviceStateChange(attribute="mode", type="config", previous_state="a", new_state="b", **ctx)
        out.append(e)
    return out


def _same(a, b):
    da, db = a.to_dict(), b.to_dict()
    da.pop("receivedDate", None)
    db.pop("receivedDate", None)
    assert da == db, (da, db)


def test_api_events_become_indexed_block_rows(tmp_path, monkeypatch):
    """Every event type added through the API round-trips through a block row exactly (ids, context,
    alternate ids, metadata, type fields), is found by id, alternate id and every index, and a
    command response by its invocation -- before and after the tail is flushed into a block."""
    monkeypatch.setenv("SW_API_FLUSH_S", "3600")
    from sitewhere_amd.models.domain import DateRangeSearchCriteria, DeviceEventType
    from sitewhere_amd.persistence.segments import DurableEventStore
    d = str(tmp_path / "s")
    st = DurableEventStore(d, direct=False)
    evs = _api_events(700)
    st.add_events(evs[:300])
    st.add_events(evs[300:])
    inv = next(e for e in evs if e.event_type == DeviceEventType.CommandInvocation)
    from sitewhere_amd.models.domain import DeviceCommandResponse
    resp = DeviceCommandResponse(originating_event_id=inv.id, response="done", device_assignment_id=inv.device_assignment_id,
                                 device_id=inv.device_id, customer_id=inv.customer_id, area_id=inv.area_id,
                                 asset_id=inv.asset_id, event_date=1_000_999)
    st.add_events([resp])
    evs.append(resp)

    def check(store):
        for e in evs[::13] + [resp]:
            _same(store.get_event_by_id(e.id), e)
        for e in evs[:60]:
            if e.alternate_id:
                assert store.get_event_by_alternate_id(e.alternate_id).id == e.id
        for ix, key, tok in (("Assignment", "device_assignment_id", "asg-3"), ("Area", "area_id", "area-1"),
                             ("Customer", "customer_id", "cust-2"), ("Asset", "asset_id", "asset-1")):
            for et in ("Measurement", "Alert", "CommandInvocation", "StateChange"):
                want = sorted((e for e in evs if getattr(e, key) == tok and e.event_type == et),
                              key=lambda e: (-e.event_date, e.id))
                r = store.list_events(et, ix, [tok], DateRangeSearchCriteria(page_size=25))
                assert r.num_results == len(want), (ix, et)
                assert [x.id for x in r.results] == [x.id for x in want[:25]], (ix, et)
        rs = store.list_command_responses_for_invocation(inv.id).results
        assert [x.id for x in rs] == [resp.id] and rs[0].response == "done"

    check(st)                                                 # from the tail
    assert st.flush_api() == 701 and not st._api_tail
    check(st)                                                 # from the block
    st.close()
    st = DurableEventStore(d, direct=False)
    try:
        check(st)
        ents = st.seg.index()
        assert len(ents) == 1 and int(ents[0]["n_rows"]) == 701 and os.path.getsize(os.path.join(d, "api-0.log")) == 0
    finally:
        st.close()


def test_api_restart_is_bounded_by_the_tail(tmp_path, monkeypatch):
    """1M API-added events: the tail is flushed into blocks as it fills, so the process's memory
    does not grow with the events added and a restart replays only the tail (its time does not
    grow with history); every event is readable after a kill."""
    import resource
    monkeypatch.setenv("SW_API_FLUSH_EVENTS", "50000")
    monkeypatch.setenv("SW_API_FLUSH_S", "0.2")
    from sitewhere_amd.persistence.segments import DurableEventStore
    d = str(tmp_path / "s")
    st = DurableEventStore(d, direct=False)
    import time
    rss = []
    first = last = None
    total = 1_000_000
    for k in range(0, total, 10_000):
        batch = _api_events(10_000, seed=k)
        st.add_events(batch)
        first = first or batch[0]
        last = batch[-1]
        if k in (200_000, 990_000):
            rss.append(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss)
    while len(st._api_tail) > 60_000:                          # the flusher keeps up
        time.sleep(0.05)
    _crash(st)
    tail = len(st._api_tail)
    t0 = time.perf_counter()
    st = DurableEventStore(d, direct=False)
    reopen = time.perf_counter() - t0
    try:
        assert len(st._api_tail) == tail
        _same(st.get_event_by_id(first.id), first)
        _same(st.get_event_by_id(last.id), last)
        assert st.count() == total
        assert rss[1] - rss[0] < 400 * 1024, rss                 # KiB: growth over the last 790K events
        assert reopen < 5.0, reopen
    finally:
        st.close()


def test_oversized_api_add_is_refused_before_the_log(tmp_path, monkeypatch):
    """an event whose metadata, alternate id or alert message does not fit a block
    row (u16 string spans) is refused by the add -- it never reaches the write-ahead log, so the tail
    keeps flushing into blocks; nothing is silently truncated (a cut alternate id would break its
    dedup); a flush failure is visible in ``retention_state``."""
    monkeypatch.setenv("SW_API_FLUSH_S", "3600")
    from sitewhere_amd.core.errors import SiteWhereSystemException
    from sitewhere_amd.models.domain import DeviceAlert, DeviceMeasurement
    from sitewhere_amd.persistence.segments import DurableEventStore
    d = str(tmp_path / "s")
    st = DurableEventStore(d, direct=False)
    try:
        ctx = dict(device_assignment_id="asg-1", device_id="dev-1", customer_id="c", area_id="a", asset_id="x",
                   event_date=1_000_000)
        bad = [DeviceMeasurement(name="t", value=1.0, metadata={"k": "v" * 70_000}, **ctx),
               DeviceMeasurement(name="t", value=1.0, alternate_id="a" * 70_000, **ctx),
               DeviceAlert(type="door", message="m" * 70_000, **ctx)]
        for e in bad:
            with pytest.raises(SiteWhereSystemException):
                st.add_events([e])
        ok = DeviceMeasurement(name="t", value=2.0, alternate_id="fine-1", metadata={"k": "v"}, **ctx)
        st.add_events([ok])
        assert len(st._api_tail) == 1
        assert st.flush_api() == 1 and not st._api_tail
        assert st.retention_state()["api_flush_error"] is None
        assert st.get_event_by_alternate_id("fine-1").id == ok.id
        assert os.path.getsize(os.path.join(d, "api-0.log")) == 0
    finally:
        st.close()


def test_alternate_hash_chunks_skip_over_mixed_block_sizes(tmp_path, monkeypatch):
    """seeding the dedup filter pages through the store's ids with ``skip``.
    Over blocks of mixed sizes, the concatenated pages equal the unpaged sequence for every page size
    (whole blocks are skipped by count only before the first block kept)."""
    import numpy as np
    monkeypatch.setenv("SW_API_FLUSH_S", "3600")
    from sitewhere_amd.models.domain import DeviceMeasurement
    from sitewhere_amd.persistence.segments import DurableEventStore
    st = DurableEventStore(str(tmp_path / "s"), direct=False)
    try:
        k = 0
        for n in (20, 5, 13, 40, 1, 9):
            evs = [DeviceMeasurement(name="t", value=float(i), alternate_id=f"alt-{k + i}", device_assignment_id="a",
                                     device_id="d", event_date=1_000_000 + k + i) for i in range(n)]
            k += n
            st.add_events(evs)
            assert st.flush_api() == n
        full = np.concatenate(list(st.alternate_hash_chunks(1 << 20)))
        assert len(full) == k == len(set(full.tolist()))
        for page in (1, 3, 7, 10, 21, 50):
            got, skip = [], 0
            while True:
                part = list(st.alternate_hash_chunks(page, skip=skip))
                h = np.concatenate(part) if part else np.zeros(0, np.uint64)
                if not len(h):
                    break
                assert len(h) <= page
                got.append(h)
                skip += len(h)
            assert np.array_equal(np.concatenate(got), full), page
    finally:
        st.close()


def test_retention_by_rows_bounds_the_store(tmp_path, monkeypatch):
    """an engine tenant bounds its durable store to the rows its dedup filter still
    holds ids for.  Whole files go, oldest first, after every group commit: the store keeps at most
    the limit plus the file being written, and never less than the limit minus one file."""
    monkeypatch.setenv("SW_API_FLUSH_S", "3600")
    from sitewhere_amd.models.domain import DeviceMeasurement
    from sitewhere_amd.persistence.segments import DurableEventStore
    st = DurableEventStore(str(tmp_path / "s"), direct=False, rotate_bytes=64 << 10)
    try:
        assert st.limit_retention_rows(3000) == 3000
        assert st.limit_retention_rows(5000) == 3000                    # only ever tightens
        k = 0
        for _ in range(40):
            st.add_events([DeviceMeasurement(name="t", value=float(i), alternate_id=f"r-{k + i}",
                                             device_assignment_id="a", device_id="d", event_date=1_000_000 + k + i)
                           for i in range(250)])
            k += 250
            assert st.flush_api() == 250
            rs = st.retention_state()
            assert rs["retained_rows"] <= 3000 + 64 * 1024 // 8, rs
        rs = st.retention_state()
        assert rs["deleted_rows"] + rs["retained_rows"] == k and rs["deleted_rows"] >= k - 3000 - 8192
        assert rs["retained_rows"] >= 3000 - 64 * 1024 // 8
        assert st.get_event_by_alternate_id(f"r-{k - 1}") is not None            # the newest are kept
        assert st.get_event_by_alternate_id("r-0") is None                      # the oldest are gone
    finally:
        st.close()
