"""Query push-down in the entity stores (``persistence/query.py``).

Reference: ``MongoDeviceManagement.java:758-773`` builds a filter per list call and
``MongoPersistence.java:157`` runs ``find(filter).skip().limit().sort()`` plus a count, so a page
costs a page.  Here ``list_devices`` / ``list_device_assignments`` page a 200K-device tenant by
device type, customer and area on SQLite and on the in-process MongoDB server (the wire-protocol
client and server of ``persistence/mongo_*.py``), and the store materialises at most one page of
documents per call (``EntityStore.loads``)."""
from __future__ import annotations

import time

import pytest

from sitewhere_amd.models.domain import Device, DeviceAssignment, DeviceAssignmentStatus
from sitewhere_amd.persistence.store import MemoryEntityStore, MongoEntityStore, SQLiteEntityStore
from sitewhere_amd.services.device_management import DeviceManagement

N = 200_000
TYPES, CUSTOMERS, AREAS = 20, 50, 8


def _populate(dm: DeviceManagement):
    types = [dm.create_device_type({"token": f"t{i}", "name": f"T{i}"}).id for i in range(TYPES)]
    devs, asgs = [], []
    t0 = 1_700_000_000_000
    for i in range(N):
        d = Device(token=f"d{i:06d}", device_type_id=types[i % TYPES], created_date=t0 + i)
        a = DeviceAssignment(token=f"a{i:06d}", device_id=d.id, device_type_id=d.device_type_id,
                             customer_id=f"cust-{i % CUSTOMERS}", area_id=f"area-{i % AREAS}",
                             status=DeviceAssignmentStatus.Active if i % 10 else DeviceAssignmentStatus.Released,
                             active_date=t0 + i, created_date=t0 + i)
        d.device_assignment_id = a.id if i % 10 else None
        devs.append(d)
        asgs.append(a)
    dm.devices.s.put_many("devices", devs)
    dm.assignments.s.put_many("assignments", asgs)
    return types


def _check(dm: DeviceManagement, types):
    s = dm.devices.s
    # devices of one type, newest first, page 3 of 25
    s.loads = 0
    r = dm.list_devices({"deviceTypeId": types[7], "pageNumber": 3, "pageSize": 25})
    assert r.num_results == N // TYPES and len(r.results) == 25 and s.loads <= 25
    want = [f"d{i:06d}" for i in range(N - TYPES + 7, -1, -TYPES)][50:75]
    assert [d.token for d in r.results] == want
    # by device type token, unassigned only
    s.loads = 0
    r = dm.list_devices({"deviceTypeToken": "t3", "excludeAssigned": True, "pageSize": 10})
    assert r.num_results == len([i for i in range(3, N, TYPES) if i % 10 == 0]) and s.loads <= 10 + 1
    assert all(d.device_assignment_id is None for d in r.results)
    # assignments by customer, by area, by customer + area (id lists, as the reference criteria carry)
    s.loads = 0
    r = dm.list_device_assignments({"customerId": "cust-7", "pageNumber": 2, "pageSize": 50})
    assert r.num_results == N // CUSTOMERS and len(r.results) == 50 and s.loads <= 50
    assert all(a.customer_id == "cust-7" for a in r.results)
    assert [a.active_date for a in r.results] == sorted((a.active_date for a in r.results), reverse=True)
    s.loads = 0
    r = dm.list_device_assignments({"areaIds": ["area-1", "area-2"], "customerIds": ["cust-3"], "status": "Active",
                                    "pageSize": 20})
    expect = [i for i in range(N) if i % AREAS in (1, 2) and i % CUSTOMERS == 3 and i % 10]
    assert r.num_results == len(expect) and s.loads <= 20
    assert [a.token for a in r.results] == [f"a{i:06d}" for i in sorted(expect, reverse=True)[:20]]
    s.loads = 0
    r = dm.list_device_assignments({"deviceTypeIds": [types[0]], "areaId": "area-4", "pageSize": 5})
    assert r.num_results == len([i for i in range(0, N, TYPES) if i % AREAS == 4]) and s.loads <= 5


@pytest.mark.parametrize("backend", ["memory", "sqlite", "mongo"])
def test_list_pages_push_down_on_200k_devices(backend, tmp_path):
    server = None
    if backend == "memory":
        store = MemoryEntityStore()
    elif backend == "sqlite":
        store = SQLiteEntityStore(str(tmp_path / "dm.db"))
    else:
        from sitewhere_amd.persistence.mongo_server import MiniMongoServer
        server = MiniMongoServer(port=0).start()
        store = MongoEntityStore(f"mongodb://{server.address}", "pushdown")
    try:
        dm = DeviceManagement(store)
        t = time.time()
        types = _populate(dm)
        load_s = time.time() - t
        t = time.time()
        _check(dm, types)
        print(f"{backend}: load {load_s:.1f}s, queries {time.time() - t:.2f}s")
    finally:
        if server is not None:
            server.stop()
