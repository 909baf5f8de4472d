"""Per-tenant capacity: the ``gpu-columnar`` template holds 65,536 devices per tenant;
``gpu-columnar-1m`` is the bench's shape.  A tenant created from it takes 1M devices in its engine
(registered in bulk, as a fleet import would) and steps payloads from all of them into its durable
store.  In this container the tenant's engine is the native CPU engine (same tables and sizing)."""
from __future__ import annotations

import os
import time

import numpy as np


def wait_until(cond, timeout=60.0, step=0.05):
    end = time.time() + timeout
    while time.time() < end:
        v = cond()
        if v:
            return v
        time.sleep(step)
    return cond()


def test_million_device_tenant(tmp_path, monkeypatch):
    monkeypatch.setenv("SITEWHERE_DATA_DIR", str(tmp_path / "data"))
    from sitewhere_amd.assembly import SiteWhereInstance
    from sitewhere_amd.pipeline.fleet import FleetSpec, fingerprints, gen_payloads, gen_tokens
    from sitewhere_amd.services.tenant_management import TENANT_TEMPLATES
    cap = TENANT_TEMPLATES["gpu-columnar"]["services"]["inbound-processing"]["capacity"]
    assert cap["max_devices"] == 65536                       # the documented per-tenant cap
    sw = SiteWhereInstance().start()
    try:
        sw.wait_for_tenant("default", 60)
        tm = sw.api("TenantManagement")
        sw.instance.system_user.run(lambda: tm.create_tenant({"token": "big", "name": "big",
                                                              "configurationTemplateId": "gpu-columnar-1m",
                                                              "datasetTemplateId": "empty"}))
        sw.wait_for_tenant("big", 120)
        ib = sw.tenant_engine("inbound-processing", "big")
        n = 1 << 20
        assert ib.engine.cfg.max_devices >= n and ib.engine.cfg.max_assignments >= n
        heap, offs = gen_tokens("dev-", 0, n)
        lo, hi = fingerprints(heap, offs)
        dev = ib.engine.register_devices(lo, hi)
        ib.engine.set_assignments(dev, dev, customer=dev % 97, area=dev % 31, asset=dev % 1009)
        assert ib.engine.n_assignments >= n
        spec = FleetSpec(prefix="dev-", n_devices=n, p_location=0.25, p_alert=0.05, with_alternate_id=True)
        raw, offs = gen_payloads(spec, 1 << 18, int(time.time() * 1000) - 1000, seed=3)
        raw = np.concatenate([raw, np.zeros(64, np.uint8)])
        res = ib.process_batch(raw, offs)
        ib.flush()
        assert res.n_persisted > 250_000
        # the rows come from devices across the whole fleet
        asg = res.out["assignment"]
        assert int(asg.max()) > n - 4096 and len(np.unique(asg)) > 200_000
        store = sw.tenant_engine("event-management", "big").store
        assert wait_until(lambda: store.engine_rows >= res.n_persisted, 60)
    finally:
        sw.stop()
