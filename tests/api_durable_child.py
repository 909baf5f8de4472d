"""Child process of ``tests/test_api_durable.py``: an instance with an engine tenant (``gpu-columnar``,
durable segment store) named ``dur``.  Adds events through the REST API (a measurement, a command
invocation and its response) and sends JSON device requests through the tenant's JSON event source
(transcoded onto the engine path), reads the JSON events back over REST, prints one JSON line with
what it saw, then dies with ``os._exit`` right after the last REST add returned (nothing flushed or
closed: a kill)."""
from __future__ import annotations

import base64
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
API = "/sitewhere/api"


def json_requests():
    def j(typ, req):
        return json.dumps({"deviceToken": "galaxytab-001", "type": typ, "request": req}).encode()
    return [j("DeviceAlert", {"type": "door.open", "message": "door opened at gate 3", "alternateId": "json-a-1",
                              "eventDate": 1_700_000_000_001, "metadata": {"gate": "3", "shift": "night"}}),
            j("DeviceMeasurement", {"name": "json.temp", "value": 21.25, "alternateId": "json-m-1",
                                    "eventDate": 1_700_000_000_002, "metadata": {"unit": "C"}}),
            j("DeviceLocation", {"latitude": 34.1, "longitude": -84.2, "elevation": 301.5, "alternateId": "json-l-1",
                                 "eventDate": 1_700_000_000_003})]


def main():
    from fastapi.testclient import TestClient

    from sitewhere_amd.assembly import SiteWhereInstance
    sw = SiteWhereInstance().start()
    sw.wait_for_tenant("default", 60)
    tm = sw.api("TenantManagement")
    sw.instance.system_user.run(lambda: tm.create_tenant({"token": "dur", "name": "dur", "authenticationToken": "dur-a",
                                                          "configurationTemplateId": "gpu-columnar",
                                                          "datasetTemplateId": "construction"}))
    sw.wait_for_tenant("dur", 60)
    client = TestClient(sw.rest_app)
    r = client.get("/sitewhere/authapi/jwt",
                   headers={"Authorization": "Basic " + base64.b64encode(b"admin:password").decode()})
    h = {"Authorization": f"Bearer {r.headers['X-Sitewhere-JWT']}", "X-SiteWhere-Tenant-Id": "dur",
         "X-SiteWhere-Tenant-Auth": "dur-a"}
    asg = client.get(f"{API}/devices/galaxytab-001/assignment", headers=h).json()["token"]
    ib = sw.tenant_engine("inbound-processing", "dur")
    dev = client.get(f"{API}/devices/galaxytab-001", headers=h).json()
    end = time.time() + 60
    while ib.asg_index.idx.get(dev["deviceAssignmentId"]) is None and time.time() < end:
        time.sleep(0.02)

    # JSON device requests -> transcoded -> engine -> durable block; read back over REST
    es = sw.tenant_engine("event-sources", "dur")
    for m in json_requests():
        es.inject("default-json", m)
    seen = {}
    end = time.time() + 60
    while len(seen) < 3 and time.time() < end:
        for alt in ("json-a-1", "json-m-1", "json-l-1"):
            if alt not in seen:
                g = client.get(f"{API}/events/alternate/{alt}", headers=h)
                if g.status_code == 200:
                    seen[alt] = g.json()
        time.sleep(0.05)
    sw.tenant_engine("event-management", "dur").store.flush()
    engine = type(ib.engine).__name__

    # REST adds: synchronous and durable when the call returns
    m = client.post(f"{API}/assignments/{asg}/measurements", headers=h,
                    json={"name": "api.temp", "value": 12.5, "eventDate": 1_700_000_000_100, "alternateId": "api-m-1",
                          "metadata": {"src": "rest"}}).json()
    inv = client.post(f"{API}/assignments/{asg}/invocations", headers=h,
                      json={"commandToken": "galaxytab-bannerMessage", "parameterValues": {"message": "hi"}}).json()
    resp = client.post(f"{API}/assignments/{asg}/responses", headers=h,
                       json={"originatingEventId": inv["id"], "response": "done", "alternateId": "api-r-1"}).json()
    print(json.dumps({"json": seen, "engine": engine, "measurement": m, "invocation": inv, "response": resp}),
          flush=True)
    os._exit(9)                                  # killed: nothing flushed, nothing closed


if __name__ == "__main__":
    main()
