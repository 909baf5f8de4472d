"""MongoDB wire protocol: BSON, the OP_MSG client (SCRAM auth), the in-process server, and the
reference's MongoDB datastores (entities + events) on top.

Parity unpinned against a real mongod (none in this environment): client and server are checked
against each other and against the published constants (BSON spec layouts, SCRAM RFC 5802/7677
message flow, E11000 duplicate-key code)."""
import datetime
import time

import pytest

from sitewhere_amd.persistence import bson
from sitewhere_amd.persistence.mongo_server import MiniMongoServer
from sitewhere_amd.persistence.mongo_wire import DUPLICATE_KEY, MongoClient, MongoError


@pytest.fixture
def mongo():
    srv = MiniMongoServer(port=0, users={"sw": "s3cret"}).start()
    yield srv
    srv.stop()


def uri(srv, db="tenant", user="sw", pw="s3cret", mech=None):
    q = "?authSource=admin" + (f"&authMechanism={mech}" if mech else "")
    return f"mongodb://{user}:{pw}@{srv.address}/{db}{q}"


def test_bson_roundtrip_and_layout():
    assert bson.encode({}) == b"\x05\x00\x00\x00\x00"
    assert bson.encode({"a": 1}) == b"\x0c\x00\x00\x00\x10a\x00\x01\x00\x00\x00\x00"     # bsonspec example shape
    doc = {"s": "héllo", "i": 7, "l": 1 << 40, "L": bson.Int64(3), "f": 2.5, "b": False, "n": None,
           "bin": b"\x00\xff", "arr": [1, "two", {"x": [3.0]}], "oid": bson.ObjectId(),
           "t": datetime.datetime(2021, 5, 6, 7, 8, 9, 123000, tzinfo=datetime.timezone.utc)}
    back = bson.decode(bson.encode(doc))
    assert back == doc and list(back) == list(doc)


def test_crud_cursors_updates_and_unique_indexes(mongo):
    c = MongoClient(uri(mongo))["tenant"]["devices"]
    c.create_index({"token": 1}, unique=True, sparse=True)
    c.insert_many([{"_id": f"d{i}", "token": f"t{i}", "n": i, "tags": ["a", "b"] if i % 2 else ["c"]}
                   for i in range(250)])
    assert c.count_documents({}) == 250
    got = c.find({"n": {"$gte": 10, "$lt": 200}, "tags": "a"}, sort={"n": -1}, skip=5, limit=50, batch_size=7)
    assert [d["n"] for d in got] == list(range(199 - 10, 9, -2))[:50]          # getMore across 8 batches
    assert c.find_one({"token": {"$in": ["t3", "zz"]}})["_id"] == "d3"
    c.update_one({"_id": "d3"}, {"$set": {"meta.zone": "z1"}, "$inc": {"n": 1000}, "$unset": {"tags": ""}})
    d3 = c.find_one({"_id": "d3"})
    assert d3["n"] == 1003 and d3["meta"] == {"zone": "z1"} and "tags" not in d3
    c.replace_one({"_id": "new"}, {"_id": "new", "token": "tn"}, upsert=True)
    assert c.find_one({"token": "tn"})["_id"] == "new"
    with pytest.raises(MongoError) as e:
        c.insert_one({"_id": "dup", "token": "t1"})
    assert e.value.code == DUPLICATE_KEY
    c.insert_many([{"_id": "x1"}, {"_id": "x2"}])                              # sparse: no token is fine
    assert c.delete_many({"n": {"$lt": 100}}) == 99                         # d3 was bumped to 1003
    assert c.count_documents({"_id": {"$in": ["x1", "x2"]}}) == 2
    c.drop()
    assert c.count_documents({}) == 0


@pytest.mark.parametrize("mech", ["SCRAM-SHA-256", "SCRAM-SHA-1"])
def test_scram_authentication(mongo, mech):
    assert MongoClient(uri(mongo, mech=mech))["tenant"]["x"].count_documents({}) == 0
    with pytest.raises(MongoError):
        MongoClient(uri(mongo, pw="nope", mech=mech))
    anon = MongoClient(f"mongodb://{mongo.address}/tenant")
    with pytest.raises(MongoError):
        anon["tenant"]["x"].count_documents({})


def test_mongo_entity_store(mongo):
    from sitewhere_amd.core.errors import SiteWhereSystemException
    from sitewhere_amd.models.domain import Device
    from sitewhere_amd.persistence.store import MongoEntityStore
    s = MongoEntityStore(uri(mongo), "tenant-a")
    s.register("devices", Device, ("token",))
    d = s.put("devices", Device(token="dev-1", device_type_id="tt", comments="first"))
    assert s.get("devices", d.id).comments == "first"
    assert s.get_by_token("devices", "dev-1").id == d.id
    d.comments = "updated"
    s.put("devices", d)
    assert s.count("devices") == 1 and s.get("devices", d.id).comments == "updated"
    with pytest.raises(SiteWhereSystemException):
        s.put("devices", Device(token="dev-1", device_type_id="tt"))
    assert [e.token for e in s.query("devices")] == ["dev-1"]
    assert s.delete("devices", d.id).token == "dev-1" and s.get("devices", d.id) is None


def test_mongo_event_store_queries(mongo):
    from sitewhere_amd.models.domain import (DateRangeSearchCriteria, DeviceCommandResponse, DeviceEventIndex,
                                             DeviceEventType, DeviceMeasurement)
    from sitewhere_amd.persistence.events import MongoEventStore
    s = MongoEventStore(uri(mongo), "tenant-a")
    evs = [DeviceMeasurement(device_assignment_id=f"a{i % 3}", customer_id="c", name="t", value=float(i),
                             event_date=1000 + i, alternate_id=f"alt-{i}") for i in range(30)]
    s.add_events(evs)
    s.add_events(evs[:5])                                   # idempotent by id (bulk upsert)
    assert s.count() == 30
    r = s.list_events(DeviceEventType.Measurement, DeviceEventIndex.Assignment, ["a1"],
                      DateRangeSearchCriteria(page_number=2, page_size=3, start_date=1005, end_date=1025))
    a1 = sorted((e.event_date for e in evs if e.device_assignment_id == "a1" and 1005 <= e.event_date <= 1025),
                reverse=True)
    assert r.num_results == len(a1) and [e.event_date for e in r.results] == a1[3:6]
    assert s.get_event_by_alternate_id("alt-7").value == 7.0
    assert s.get_event_by_id(evs[2].id).device_assignment_id == "a2"
    resp = DeviceCommandResponse(originating_event_id="inv-1", response="ok", event_date=5)
    s.add_events([resp])
    assert s.list_command_responses_for_invocation("inv-1").results[0].response == "ok"


def test_tenant_on_the_mongodb_template(mongo, monkeypatch):
    """A tenant created from the ``mongodb`` template keeps devices and events in MongoDB."""
    from sitewhere_amd.assembly import SiteWhereInstance
    from sitewhere_amd.models import wire
    monkeypatch.setenv("MONGODB_URI", uri(mongo, db="admin"))
    sw = SiteWhereInstance().start()
    try:
        sw.wait_for_tenant("default", 60)
        tm = sw.api("TenantManagement")
        sw.instance.system_user.run(lambda: tm.create_tenant({"token": "mg", "name": "mg",
                                                              "configurationTemplateId": "mongodb",
                                                              "datasetTemplateId": "construction"}))
        sw.wait_for_tenant("mg", 120)
        run = lambda f: sw.instance.system_user.run(f, "mg")  # noqa: E731
        dm, em = sw.api("DeviceManagement", "mg"), sw.api("DeviceEventManagement", "mg")
        dev = run(lambda: dm.get_device_by_token("meitrack-000"))
        sw.tenant_engine("event-sources", "mg").inject("default-protobuf",
                                                        wire.measurements("meitrack-000", {"mongo.t": 4.5}))
        end, res = time.time() + 30, []
        while not res and time.time() < end:
            res = run(lambda: em.list_measurements_for_index("Assignment", [dev.device_assignment_id])).results
            time.sleep(0.1)
        assert res and res[0].value == 4.5
        db = MongoClient(uri(mongo, db="admin"))["tenant-mg"]
        assert db["devices"].find_one({"token": "meitrack-000"}) is not None
        assert db["events"].count_documents({"eventType": "Measurement"}) >= 1
    finally:
        sw.stop()
