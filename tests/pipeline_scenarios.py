"""Shared scenario builders for the pipeline-engine tests (CPU oracle and GPU engine)."""
import numpy as np

from sitewhere_amd.models import wire
from sitewhere_amd.pipeline.config import EngineConfig
from sitewhere_amd.pipeline.engine_base import Zone, ZoneTest
from sitewhere_amd.pipeline.fleet import gen_tokens, fingerprints, gen_payloads, FleetSpec, pack_messages

NOW = 1_700_000_000_000
SQUARE = [(33.0, -85.0), (33.0, -84.0), (34.0, -84.0), (34.0, -85.0)]


def setup_fleet(engine, n_dev=1000, prefix="dev-", unassigned_every=10):
    heap, offs = gen_tokens(prefix, 0, n_dev)
    lo, hi = fingerprints(heap, offs)
    engine.register_devices(lo, hi)
    dev = np.arange(n_dev, dtype=np.int32)
    active = (dev % unassigned_every != unassigned_every - 1).astype(np.uint8)
    engine.set_assignments(dev, dev, customer=dev % 7, area=dev % 5, asset=dev % 3, active=active)
    engine.set_zone_rules([Zone("z1", SQUARE)], [ZoneTest("z1", "inside", "zone.enter", 2),
                                                 ZoneTest("z1", "outside", "zone.exit", 1)])
    return lo, hi


def small_cfg(**kw):
    return EngineConfig.small(**kw)


def hand_batch():
    """A hand-written batch covering every validation outcome."""
    msgs = [
        wire.measurements("dev-0000000001", {"temp": 20.0, "hum": 50.0}, event_date=NOW - 100),
        wire.measurements("dev-0000000001", {"temp": 21.0}, event_date=NOW - 50),
        wire.measurements("dev-0000000001", {"temp": 19.0}, event_date=NOW - 500),   # older: not last
        wire.location("dev-0000000002", 33.5, -84.5, event_date=NOW - 10),          # inside z1
        wire.location("dev-0000000003", 10.0, 10.0, event_date=NOW - 10),           # outside z1
        wire.alert("dev-0000000004", "overheat", "too hot", NOW - 5),
        wire.location("dev-0000000009", 33.5, -84.5),                               # unassigned (9 % 10 == 9)
        wire.location("nope-unknown", 1.0, 1.0),                                    # unregistered
        wire.location("dev-0000000005", 1.0, 1.0, alternate_id="A"),
        wire.location("dev-0000000005", 1.0, 1.0, alternate_id="A"),                # duplicate in batch
        wire.registration("dev-new", "tt"),                                         # control
        b"\x01\x00garbage",                                                         # decode error
    ]
    return pack_messages(msgs)


def fleet_batch(n_msgs, seed, n_dev=1000, **kw):
    spec = FleetSpec(prefix="dev-", n_devices=n_dev, p_location=0.3, p_alert=0.1, p_unregistered=0.02,
                     mx_per_msg=2, n_names=8, with_alternate_id=True, lat0=32.8, lon0=-85.2, span_deg=1.5, **kw)
    raw, offs = gen_payloads(spec, n_msgs, NOW - 60_000, seed)
    return np.concatenate([raw, np.zeros(64, np.uint8)]), offs


def canon_out(out, names):
    """Order-independent view of outbound rows (event ids of generated rows are order dependent)."""
    rows = []
    for r in out:
        rows.append((int(r["etype"]), int(r["assignment"]), int(r["event_date"]),
                     round(float(r["v0"]), 9), round(float(r["v1"]), 9), int(r["level"])))
    return sorted(rows)
