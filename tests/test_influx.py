"""InfluxDB event store: line-protocol writes + the reference's InfluxQL reads
(``InfluxDbDeviceEvent.java`` queries) against the in-process InfluxDB 1.x API stand-in.
Parity unpinned against a real influxd (none here)."""
import time

from sitewhere_amd.models.domain import (DateRangeSearchCriteria, DeviceAlert, DeviceCommandResponse, DeviceEventIndex,
                                         DeviceEventType, DeviceLocation, DeviceMeasurement)
from sitewhere_amd.persistence.events import InfluxEventStore
from sitewhere_amd.persistence.influx_server import MiniInfluxServer, parse_line


def test_line_protocol_parser_escapes():
    m, tags, fields, ts = parse_line(r'events,type=Alert,area=north\ wing eid="e1",doc="{\"m\":\"a,b c\"}",n=3i,x=1.5 1700',
                                     "ms")
    assert (m, ts) == ("events", 1700)
    assert tags == {"type": "Alert", "area": "north wing"}
    assert fields == {"eid": "e1", "doc": '{"m":"a,b c"}', "n": 3, "x": 1.5}


def test_influx_event_store_reference_queries():
    srv = MiniInfluxServer(port=0).start()
    try:
        s = InfluxEventStore(srv.url, "tenant-a")
        evs = [DeviceMeasurement(device_assignment_id=f"a{i % 3}", customer_id="c1", name="temp", value=float(i),
                                 event_date=1000 + i, alternate_id=f"alt-{i}") for i in range(30)]
        evs.append(DeviceLocation(device_assignment_id="a1", latitude=33.5, longitude=-84.25, event_date=2000))
        evs.append(DeviceAlert(device_assignment_id="a1", type="overheat", message='hot, "very"', event_date=2001))
        s.add_events(evs)
        assert s.count() == 32
        c = DateRangeSearchCriteria(page_number=2, page_size=3, start_date=1005, end_date=1025)
        r = s.list_events(DeviceEventType.Measurement, DeviceEventIndex.Assignment, ["a1", "a2"], c)
        want = sorted((e.event_date for e in evs[:30] if e.device_assignment_id in ("a1", "a2")
                       and 1005 <= e.event_date <= 1025), reverse=True)
        assert r.num_results == len(want) and [e.event_date for e in r.results] == want[3:6]
        assert all(e.name == "temp" for e in r.results)
        assert s.get_event_by_alternate_id("alt-7").value == 7.0
        assert s.get_event_by_id(evs[30].id).latitude == 33.5
        al = s.list_events(DeviceEventType.Alert, DeviceEventIndex.Customer, ["nobody"])
        assert al.num_results == 0
        assert s.list_events(DeviceEventType.Alert, DeviceEventIndex.Assignment, ["a1"]).results[0].message == 'hot, "very"'
        s.add_events([DeviceCommandResponse(originating_event_id="inv-9", response="done", event_date=3000)])
        assert s.list_command_responses_for_invocation("inv-9").results[0].response == "done"
    finally:
        srv.stop()


def test_tenant_on_the_influxdb_template(monkeypatch):
    from sitewhere_amd.assembly import SiteWhereInstance
    from sitewhere_amd.models import wire
    srv = MiniInfluxServer(port=0).start()
    monkeypatch.setenv("INFLUXDB_URL", srv.url)
    sw = SiteWhereInstance().start()
    try:
        sw.wait_for_tenant("default", 60)
        tm = sw.api("TenantManagement")
        sw.instance.system_user.run(lambda: tm.create_tenant({"token": "fx", "name": "fx",
                                                              "configurationTemplateId": "influxdb",
                                                              "datasetTemplateId": "construction"}))
        sw.wait_for_tenant("fx", 120)
        run = lambda f: sw.instance.system_user.run(f, "fx")  # noqa: E731
        dm, em = sw.api("DeviceManagement", "fx"), sw.api("DeviceEventManagement", "fx")
        aid = run(lambda: dm.get_device_by_token("meitrack-000")).device_assignment_id
        sw.tenant_engine("event-sources", "fx").inject("default-protobuf",
                                                        wire.measurements("meitrack-000", {"influx.t": 2.5}))
        end, res = time.time() + 30, []
        while not res and time.time() < end:
            res = run(lambda: em.list_measurements_for_index("Assignment", [aid])).results
            time.sleep(0.1)
        assert res and res[0].value == 2.5
        assert srv.query("tenant-fx", "SELECT count(eid) FROM events WHERE type='Measurement'")["series"][0]["values"][0][1] >= 1
    finally:
        sw.stop()
        srv.stop()
