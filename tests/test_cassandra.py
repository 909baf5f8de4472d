"""Cassandra: the CQL native protocol v4 client, the in-process CQL server, and the event store in
the reference's bucketed table layout.  Parity unpinned against a real Cassandra (none here): client
and server are checked against each other and the protocol's frame/notation layouts."""
import time

import pytest

from sitewhere_amd.persistence.cql_server import MiniCassandraServer
from sitewhere_amd.persistence.cql_wire import CqlError, CqlSession


@pytest.fixture
def cass():
    srv = MiniCassandraServer(port=0, users={"cassandra": "pw"}).start()
    yield srv
    srv.stop()


def test_cql_ddl_prepared_inserts_and_clustered_reads(cass):
    s = CqlSession(cass.address, username="cassandra", password="pw")
    s.execute("CREATE KEYSPACE IF NOT EXISTS ks WITH replication = {'class': 'SimpleStrategy', 'replication_factor': 1}")
    s.execute("USE ks")
    s.execute("CREATE TABLE t (a text, b tinyint, c int, d timestamp, e text, v double, ok boolean, "
              "PRIMARY KEY ((a, b, c), d, e)) WITH CLUSTERING ORDER BY (d DESC, e ASC)")
    for i in range(20):
        s.execute("INSERT INTO t (a, b, c, d, e, v, ok) VALUES (?, ?, ?, ?, ?, ?, ?)",
                  ["x", 1, i % 2, 1000 + i, f"id{i:02d}", i * 0.5, i % 3 == 0])
    s.execute("INSERT INTO t (a, b, c, d, e, v) VALUES (?, ?, ?, ?, ?, ?)", ["x", 1, 0, 1000, "id00", 99.0])  # upsert
    rows = s.execute("SELECT d, e, v FROM t WHERE a = ? AND b = ? AND c = ? AND d >= ? AND d <= ?",
                     ["x", 1, 0, 1002, 1012])
    assert [r["d"] for r in rows] == [1012, 1010, 1008, 1006, 1004, 1002]          # clustering DESC
    assert s.execute("SELECT COUNT(*) FROM t WHERE a = ? AND b = ? AND c IN (?, ?)", ["x", 1, 0, 1])[0]["count"] == 20
    assert s.execute("SELECT v, ok FROM t WHERE a = ? AND b = ? AND c = ? LIMIT 1", ["x", 1, 0])[0] == \
        {"v": 9.0, "ok": True}                                                  # i = 18
    assert s.execute("SELECT v FROM t WHERE a = ? AND b = ? AND c = ? AND d = ?", ["x", 1, 0, 1000])[0]["v"] == 99.0
    with pytest.raises(CqlError):
        s.execute("SELECT * FROM missing WHERE a = ?", ["x"])
    with pytest.raises(CqlError):
        CqlSession(cass.address, username="cassandra", password="wrong")
    s.close()


def test_cassandra_event_store_across_buckets(cass):
    from sitewhere_amd.models.domain import (DateRangeSearchCriteria, DeviceCommandResponse, DeviceEventIndex,
                                             DeviceEventType, DeviceLocation, DeviceMeasurement)
    from sitewhere_amd.persistence.events import CassandraEventStore
    s = CassandraEventStore(cass.address, "tenant-a", bucket_ms=10, username="cassandra", password="pw")
    evs = [DeviceMeasurement(device_assignment_id=f"a{i % 2}", area_id="ar", name="t", value=float(i),
                             event_date=100 + 3 * i, alternate_id=f"alt-{i}") for i in range(40)]   # ~12 buckets
    s.add_events(evs)
    s.add_events(evs[:3])                                 # re-delivery: upserts, count unchanged
    assert s.count() == 40
    r = s.list_events(DeviceEventType.Measurement, DeviceEventIndex.Assignment, ["a0"],
                      DateRangeSearchCriteria(page_number=2, page_size=4, start_date=130, end_date=200))
    want = sorted((e.event_date for e in evs if e.device_assignment_id == "a0" and 130 <= e.event_date <= 200),
                  reverse=True)
    assert r.num_results == len(want) and [e.event_date for e in r.results] == want[4:8]
    allr = s.list_events(DeviceEventType.Measurement, DeviceEventIndex.Area, ["ar"], DateRangeSearchCriteria(page_size=0))
    assert allr.num_results == 40 and allr.results[0].event_date == 217
    assert s.list_events(DeviceEventType.Location, DeviceEventIndex.Area, ["ar"]).num_results == 0
    s.add_events([DeviceLocation(device_assignment_id="a1", latitude=1.0, longitude=2.0, event_date=500)])
    assert s.list_events(DeviceEventType.Location, DeviceEventIndex.Assignment, ["a1"]).results[0].longitude == 2.0
    assert s.get_event_by_alternate_id("alt-9").value == 9.0 and s.get_event_by_id(evs[5].id).value == 5.0
    s.add_events([DeviceCommandResponse(originating_event_id="inv", response="r1", event_date=7)])
    assert s.list_command_responses_for_invocation("inv").results[0].response == "r1"


def test_tenant_on_the_cassandra_template(cass, monkeypatch):
    from sitewhere_amd.assembly import SiteWhereInstance
    from sitewhere_amd.models import wire
    srv = MiniCassandraServer(port=0).start()             # no auth: the template passes none
    monkeypatch.setenv("CASSANDRA_ADDRESS", srv.address)
    sw = SiteWhereInstance().start()
    try:
        sw.wait_for_tenant("default", 60)
        tm = sw.api("TenantManagement")
        sw.instance.system_user.run(lambda: tm.create_tenant({"token": "cq", "name": "cq",
                                                              "configurationTemplateId": "cassandra",
                                                              "datasetTemplateId": "construction"}))
        sw.wait_for_tenant("cq", 120)
        run = lambda f: sw.instance.system_user.run(f, "cq")  # noqa: E731
        dm, em = sw.api("DeviceManagement", "cq"), sw.api("DeviceEventManagement", "cq")
        aid = run(lambda: dm.get_device_by_token("meitrack-000")).device_assignment_id
        sw.tenant_engine("event-sources", "cq").inject("default-protobuf",
                                                        wire.measurements("meitrack-000", {"cql.t": 1.5}))
        end, res = time.time() + 30, []
        while not res and time.time() < end:
            res = run(lambda: em.list_measurements_for_index("Assignment", [aid])).results
            time.sleep(0.1)
        assert res and res[0].value == 1.5
        s = CqlSession(srv.address, "tenant_cq")
        assert s.execute("SELECT COUNT(*) FROM events_by_id")[0]["count"] >= 1
    finally:
        sw.stop()
        srv.stop()
