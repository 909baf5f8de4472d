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


def test_api_log_torn_tail_is_cut(tmp_path):
    """A crash mid-append leaves a partial line: reopening drops it and keeps every whole event."""
    from sitewhere_amd.models.domain import DeviceMeasurement
    from sitewhere_amd.persistence.segments import DurableEventStore
    d = str(tmp_path / "s")
    st = DurableEventStore(d, direct=False)
    evs = [DeviceMeasurement(id=f"e{i}", name="t", value=float(i), event_date=1000 + i, device_assignment_id="a1",
                             alternate_id=f"alt-{i}") for i in range(5)]
    st.add_events(evs[:3])
    st.add_events(evs[3:])
    st.close()
    path = os.path.join(d, "api-0.log")
    size = os.path.getsize(path)
    with open(path, "r+b") as f:
        f.truncate(size - 7)                  # tear the last event's line
    st = DurableEventStore(d, direct=False)
    try:
        assert [st.get_event_by_id(f"e{i}") is not None for i in range(5)] == [True] * 4 + [False]
        assert os.path.getsize(path) < size - 7              # the torn line itself was cut off
        st.add_events([evs[4]])
    finally:
        st.close()
    st = DurableEventStore(d, direct=False)
    try:
        assert st.get_event_by_alternate_id("alt-4").value == 4.0 and st.count() == 5
    finally:
        st.close()
