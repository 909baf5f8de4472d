"""Checkpoint / resume of an engine shard (registry mirror, device state, dedup window, names,
cursors, statistics, optionally the HBM event ring).

Reference: state survives a restart through Kafka offsets committed after processing
and the durable stores.  Here the hot state of a tenant lives in HBM, so a shard is snapshotted to
one safetensors file (no pickle -- loading executes nothing) and the raw-payload consumer commits
its offsets only once a snapshot covering them is on disk.  Replaying the batches after the
snapshot then reproduces exactly the same event ids, state and outputs (the engine is
deterministic), which makes the event-store sink idempotent by batch key
(``persistence/columnar.ColumnarEventStore``).

File layout: tensors ``host/*`` (registry mirror, assignment context), ``eng/*`` (engine tables,
engine-kind specific) and JSON metadata ``meta`` (config digest, counters, names, zone rules,
caller extras).
"""
from __future__ import annotations

import json
import os
from dataclasses import asdict

import numpy as np

FORMAT = "sitewhere-amd.engine-checkpoint/1"
HOST_ARRAYS = ("reg_lo", "reg_hi", "reg_val", "dev_slot", "dev_asg", "dev_type", "asg_device", "asg_customer",
               "asg_area", "asg_asset", "asg_active")
# sizes that must match between the writer and the restoring engine
SHAPE_KEYS = ("max_msgs", "rec_cap", "gen_cap", "max_devices", "max_assignments", "store_cap", "dedup_slots",
              "name_slots", "state_slots", "names_cap", "reg_slots", "shuf_cap", "carry_cap", "rank", "world")


def _shape(cfg) -> dict:
    d = asdict(cfg)
    d["reg_slots"], d["shuf_cap"] = cfg.reg_slots, cfg.shuf_cap
    return {k: int(d[k]) for k in SHAPE_KEYS}


def save_engine(engine, path: str, include_store: bool = False, extra: dict | None = None) -> int:
    """Snapshot ``engine`` to ``path`` (atomic rename).  Returns the file size in bytes."""
    from safetensors.numpy import save_file

    with engine._lock:
        tensors = {f"host/{k}": np.ascontiguousarray(getattr(engine, k)) for k in HOST_ARRAYS}
        for k, v in engine.checkpoint_state(include_store).items():
            tensors[f"eng/{k}"] = np.ascontiguousarray(v)
        meta = {
            "format": FORMAT, "kind": engine.kind, "shape": _shape(engine.cfg), "include_store": include_store,
            "n_devices": engine.n_devices, "n_assignments": engine.n_assignments, "batch_seq": engine.batch_seq,
            "presence_enabled": engine.presence_enabled, "last_presence_check": engine._last_presence_check,
            "names": {str(h): s for h, s in engine.names.items()},
            "zones": [[z.token, [list(map(float, v)) for v in z.vertices]] for z in engine.zones],
            "tests": [[t.zone_token, t.condition, t.alert_type, int(t.alert_level), t.alert_message]
                      for t in engine.tests],
            "extra": extra or {},
        }
    tmp = f"{path}.tmp-{os.getpid()}"
    save_file(tensors, tmp, metadata={"meta": json.dumps(meta)})
    os.replace(tmp, path)
    return os.path.getsize(path)


def read_meta(path: str) -> dict:
    from safetensors import safe_open
    with safe_open(path, "np") as f:
        return json.loads(f.metadata()["meta"])


def load_engine(engine, path: str) -> dict:
    """Restore a snapshot written by :func:`save_engine` into a freshly built engine of the same
    kind and sizing.  Returns the metadata ``extra`` dict the writer attached."""
    from safetensors.numpy import load_file

    from .engine_base import Zone, ZoneTest

    meta = read_meta(path)
    if meta.get("format") != FORMAT:
        raise ValueError(f"{path}: not an engine checkpoint")
    if meta["kind"] != engine.kind:
        raise ValueError(f"checkpoint of a {meta['kind']} engine cannot restore a {engine.kind} engine")
    if meta["shape"] != _shape(engine.cfg):
        diff = {k: (v, _shape(engine.cfg)[k]) for k, v in meta["shape"].items() if _shape(engine.cfg)[k] != v}
        raise ValueError(f"checkpoint sizing differs from this engine: {diff}")
    arrays = load_file(path)
    with engine._lock:
        for k in HOST_ARRAYS:
            getattr(engine, k)[...] = arrays[f"host/{k}"]
        engine.n_devices, engine.n_assignments = int(meta["n_devices"]), int(meta["n_assignments"])
        engine.batch_seq = int(meta["batch_seq"])
        engine.presence_enabled = bool(meta["presence_enabled"])
        engine._last_presence_check = meta["last_presence_check"]
        engine.names = {int(h): s for h, s in meta["names"].items()}
        zones = [Zone(tok, [tuple(v) for v in verts]) for tok, verts in meta["zones"]]
        tests = [ZoneTest(*t) for t in meta["tests"]]
        engine.set_zone_rules(zones, tests)
        engine.restore_state({k[4:]: v for k, v in arrays.items() if k.startswith("eng/")},
                             bool(meta["include_store"]))
    return meta.get("extra", {})
