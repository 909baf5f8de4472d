"""Enriched-event consumers on an engine tenant's batches: sustained events/s of
  * an MQTT outbound connector behind an area filter (and an event-type filter), publishing each
    kept event as JSON to an in-process MQTT broker (QoS 0), on its delivery pool, and
  * a threshold rule processor (measurement ``temp`` above a bound -> one batched alert add per
    batch into a durable event store: the API path, ``DeviceEventManagement.add_alert_batch``),
each fed the same engine batches (durable blocks with dictionary deltas, what an engine tenant
publishes on ``inbound-enriched-batches``: native CPU engine steps of the bench fleet).

Rates count every row of the batches the consumer processed (what it must keep up with), per
second of its own processing; ``delivered`` / ``alerts`` what passed.  Prints one JSON line."""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class _Rec:
    def __init__(self, value):
        self.value, self.key = value, None


class _Tenant:
    token = "soak"


class Area:
    """An area filter whose area id is the dictionary's area string (no device management here)."""
    def __new__(cls, engine, token, op):
        from sitewhere_amd.services.outbound_connectors import AreaFilter

        class _Area(AreaFilter):
            def area_id(self):
                return token
        return _Area(engine, token, op)


def _broker_proc(conn):
    """Child process: an MQTT broker and a subscriber to ``soak/#`` counting the messages it gets;
    sends the port, then the count when asked (after the publisher stopped and the socket drained)."""
    import time as _t
    from sitewhere_amd.edges.mqtt import MqttBroker, MqttClient
    broker = MqttBroker().start()
    got = [0]
    sub = MqttClient("127.0.0.1", broker.port).connect()
    sub.on_messages(lambda t, ps: got.__setitem__(0, got[0] + len(ps)))
    sub.subscribe("soak/#", 0)
    conn.send(broker.port)
    conn.recv()
    last, t0 = -1, _t.time()
    while got[0] != last and _t.time() - t0 < 60:      # wait until deliveries stop arriving
        last = got[0]
        _t.sleep(0.5)
    conn.send(got[0])
    sub.disconnect()
    broker.stop()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--msgs", type=int, default=1 << 16, help="payloads per batch")
    ap.add_argument("--devices", type=int, default=1 << 16)
    ap.add_argument("--batches", type=int, default=8)
    ap.add_argument("--areas", type=int, default=31)
    ap.add_argument("--threads", type=int, default=4, help="connector delivery pool")
    ap.add_argument("--seconds", type=float, default=20.0, help="per consumer")
    a = ap.parse_args()
    from sitewhere_amd.models.domain import DeviceAlert
    from sitewhere_amd.persistence.segments import DurableEventStore, encode_durable_batch, seal
    from sitewhere_amd.pipeline.config import EngineConfig
    from sitewhere_amd.pipeline.fleet import FleetSpec, fingerprints, gen_payloads, gen_tokens, hash64
    from sitewhere_amd.pipeline.native_engine import NativeCpuEngine
    from sitewhere_amd.services.enriched_batches import EnrichedBatchReader
    from sitewhere_amd.services.outbound_connectors import EventTypeFilter, MqttConnector
    from sitewhere_amd.services.rule_processing import ThresholdRuleProcessor

    # ---- engine batches of the bench fleet (native engine), with their dictionary deltas
    cfg = EngineConfig(max_msgs=a.msgs, rec_cap=2 * a.msgs, gen_cap=a.msgs, max_devices=a.devices + 1024,
                       max_assignments=a.devices + 1024, store_cap=1 << 20, dedup_slots=1 << 22, name_slots=1 << 12,
                       state_slots=1 << 20)
    eng = NativeCpuEngine(cfg)
    heap, offs = gen_tokens("dev-", 0, a.devices)
    lo, hi = fingerprints(heap, offs)
    dev = eng.register_devices(lo, hi)
    eng.set_assignments(dev, dev, customer=dev % 97, area=dev % a.areas, asset=dev % 1009)
    spec = FleetSpec(prefix="dev-", n_devices=a.devices, p_location=0.25, p_alert=0.05, p_unregistered=0.005,
                     with_alternate_id=True, lat0=33.0, lon0=-85.0, span_deg=2.0, p_meta=0.1, n_names=4)
    boot = 0x17000
    asg = {int(i): [f"asg-{i}", f"dev-{i}", f"cust-{i % 97}", f"area-{i % a.areas}", f"asset-{i % 1009}",
                    f"dev-{i}", f"type-{i % 3}"] for i in dev.tolist()}
    now = 1_700_000_000_000
    recs, rows = [], 0
    for b in range(a.batches):
        raw, off = gen_payloads(spec, a.msgs, now + 1000 * b - 30_000, seed=b + 1)
        raw = np.concatenate([raw, np.zeros(64, np.uint8)])
        res = eng.step(raw, off, now + 1000 * b, presence=False)
        blk = eng.encode_block(now + 1000 * b, res, boot=boot)
        seal(blk, rows, now + 1000 * b, boot, 0, 1)
        # the fleet's names ("mx.metric<k>", "alert.type<k>") by their interned ids
        byhash = {hash64(x): x for x in [f"mx.metric{k}" for k in range(16)] + [f"alert.type{k}" for k in range(8)]}
        names = {int(i): byhash[h] for h, i in eng.intern_table().items() if h in byhash}
        if b == 0:        # the assignment contexts travel once, ahead of the cycled batches
            prime = _Rec(encode_durable_batch(blk, boot, asg=asg, names=names))
        recs.append(_Rec(encode_durable_batch(blk, boot, names=names)))
        rows += res.n_persisted
    per_batch = rows / a.batches
    out = {"bench": "consumers", "rows_per_batch": round(per_batch), "batches": a.batches, "threads": a.threads}

    def soak(fn, seconds):
        fn([prime])
        n = k = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            fn([recs[k % len(recs)]])
            n += 1
            k += 1
        return n, time.perf_counter() - t0

    # ---- MQTT connector behind column filters, publishing to a broker in its own process (with the
    # subscriber that counts what arrives): (a) an area filter + event types (~3% of rows kept), (b)
    # event types only (~95% kept: the delivery path's throughput)
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    for name, filters in (("mqtt_area_filter", lambda: [Area(None, "area-3", "include"),
                                                        EventTypeFilter(["Measurement", "Location"])]),
                          ("mqtt_event_type_filter", lambda: [EventTypeFilter(["Measurement", "Location"])])):
        parent, child = ctx.Pipe()
        proc = ctx.Process(target=_broker_proc, args=(child,), daemon=True)
        proc.start()
        if not parent.poll(120):
            raise RuntimeError("broker process did not start")
        port = parent.recv()
        te = type("E", (), {"tenant": _Tenant()})()
        mq = MqttConnector("mq", "127.0.0.1", port, topic="soak/{tenant}/{eventType}", qos=0, filters=filters())
        mq.tenant_engine = te
        mq.set_threads(a.threads)
        mq.start(None)
        reader = EnrichedBatchReader(None)
        n, dt = soak(lambda r: mq.process_records(reader, r), a.seconds)
        mq.stop(None)
        parent.send("count")
        got = parent.recv() if parent.poll(120) else None
        proc.join(10)
        out[name] = {"events_per_s": round(n * per_batch / dt, 1), "batches": n, "seconds": round(dt, 2),
                     "delivered": mq.delivered, "filtered": mq.filtered, "received_by_subscriber": got,
                     "delivered_per_s": round(mq.delivered / dt, 1)}

    # ---- threshold rule -> batched alerts into a durable store (the API add path): a rare bound
    # (~0.01% of the rule's rows: the scan rate) and a frequent one (~5%: the alert add path)
    for name, bound in (("threshold_rule_rare", 999.9), ("threshold_rule", 950.0)):
        d = tempfile.mkdtemp(prefix="sw-soak-")
        st = DurableEventStore(d, direct=False)
        alerts = [0]

        class Api:
            def add_alert_batch(self, pairs):
                evs = [DeviceAlert(device_assignment_id=aid, type=r["type"], message=r["message"], source="System",
                                   event_date=now) for aid, r in pairs]
                st.add_events(evs)
                alerts[0] += len(evs)
        thr = ThresholdRuleProcessor("thr", [{"measurement": "mx.metric0", "max": bound, "alertType": "hot"}])
        thr.events_api = lambda: Api()
        reader2 = EnrichedBatchReader(None)
        n, dt = soak(lambda r: thr.process_records(reader2, r), a.seconds)
        out[name] = {"events_per_s": round(n * per_batch / dt, 1), "batches": n, "seconds": round(dt, 2),
                     "alerts": alerts[0], "alerts_per_s": round(alerts[0] / dt, 1)}
        st.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
