"""Child process of ``tests/test_durable_tenant.py``: one SiteWhere instance over a durable bus, with
an MI355X-pipeline tenant (``gpu-columnar``: durable segment store) named ``dur``.

``run``: publish the raw batches, then die with ``os._exit`` (no flush, no close -- a kill) once the
raw consumer has committed ``kill_after`` batches.  ``resume``: a new instance over the same
directories; waits until every batch is consumed, then stops cleanly.  Prints one JSON line with
the raw consumer group and topic before doing anything else."""
from __future__ import annotations

import json
import os
import struct
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def raw_batch(b: int, n: int):
    from sitewhere_amd.models import wire
    msgs = [wire.measurements("galaxytab-001", {"v": float(1000 * b + i)}, event_date=1_700_000_000_000 + 1000 * b + i,
                              alternate_id=f"k-{b}-{i}") for i in range(n)]
    return struct.pack(f"<I{len(msgs)}I", len(msgs), *[len(m) for m in msgs]) + b"".join(msgs)


def main():
    phase, bus_dir, n_batches, per, kill_after = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), \
        int(sys.argv[5])
    from sitewhere_amd.assembly import SiteWhereInstance
    from sitewhere_amd.bus.log import EventBus
    from sitewhere_amd.runtime.config import InstanceSettings
    from sitewhere_amd.runtime.microservice import Instance
    from sitewhere_amd.services.event_sources import RAW_PAYLOADS

    bus = EventBus(bus_dir, default_partitions=1)
    sw = SiteWhereInstance(instance=Instance(InstanceSettings.from_env(heartbeat_s=5.0), bus=bus)).start()
    sw.wait_for_tenant("default", 60)
    tm = sw.api("TenantManagement")
    sw.instance.system_user.run(lambda: tm.create_tenant({"token": "dur", "name": "dur",
                                                          "configurationTemplateId": "gpu-columnar",
                                                          "datasetTemplateId": "construction"}))
    sw.wait_for_tenant("dur", 60)
    ib = sw.tenant_engine("inbound-processing", "dur")
    topic = sw.instance.naming.tenant_prefix("dur") + RAW_PAYLOADS
    group = ib.raw_consumer.group
    print(json.dumps({"group": group, "topic": topic, "src_topic": ib._src_topic(topic), "boot": ib.boot}), flush=True)
    dev = sw.instance.system_user.run(lambda: sw.api("DeviceManagement", "dur").get_device_by_token("galaxytab-001"),
                                      "dur")
    end = time.time() + 60
    while ib.asg_index.idx.get(dev.device_assignment_id) is None and time.time() < end:
        time.sleep(0.02)
    if phase == "run":
        ib.raw_consumer.max_records = 1             # one batch per poll: the kill lands between batches
        # bus commits past kill_after are lost (as with a volatile bus, or a crash between the disk
        # and the commit): the disk then runs ahead of the bus, and the restart must trust the disk
        orig = bus.commit

        def lagging(g, t, p, o):
            if not (g == group and o > kill_after):
                orig(g, t, p, o)
        bus.commit = lagging
        store = sw.tenant_engine("event-management", "dur").store
        for b in range(n_batches):
            bus.append(topic, 0, [(None, raw_batch(b, per))], ts=1_700_000_100_000 + b)
        end = time.time() + 120
        while (store.source_offset(ib._src_topic(topic), 0) or 0) < kill_after + 3 and time.time() < end:
            time.sleep(0.001)
        os._exit(9)                                 # killed: nothing flushed, nothing closed
    end = time.time() + 120
    while bus.committed(group, topic, 0) < n_batches and time.time() < end:
        time.sleep(0.02)
    ib.flush()
    print(json.dumps({"committed": bus.committed(group, topic, 0),
                      "persisted": ib.engine.stats_dict()["persisted"]}), flush=True)
    sw.stop()


if __name__ == "__main__":
    main()
