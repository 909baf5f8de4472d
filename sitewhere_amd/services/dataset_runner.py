"""Dataset templates: initializer scripts run when a tenant is bootstrapped.

Reference: ``service-tenant-management/dockerimage/datasets/<id>/dataset-template.json`` lists, per
microservice, the Groovy initializers the tenant engine runs on bootstrap
(``initializers.deviceManagement: [initializer/deviceModel.groovy]``, ...), each bound to a builder.

Here a dataset is ``sitewhere_amd/datasets/<id>/dataset.json`` + Python initializer scripts.  A
tenant engine runs the scripts of its section with the builders bound (``device_builder``,
``event_builder``, ``asset_builder``, ``schedule_builder``) plus ``logger``, ``rnd`` (a seeded
``random.Random``), ``params`` (dataset sizing; ``SITEWHERE_DATASET_<NAME>`` overrides) and
``geo`` (point-in-polygon helpers).  A script stored in the script manager for the tenant and this
microservice under ``initializer-<name>`` (any version made active) replaces the packaged one --
the versioned user initializers of the reference.  Scripts run with the restricted builtins of
``runtime/scripting.py`` and its source check, in-process, as trusted tenant-administrator code
(they drive the management APIs directly; see that module's trust model)."""
from __future__ import annotations

import json
import logging
import os
import random

DATASET_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "datasets")

PARAM_DEFAULTS = {"devices_per_site": 30, "measurements_per_assignment": 50, "locations_per_assignment": 40,
                  "min_temp": 80, "warn_temp": 160, "error_temp": 180, "critical_temp": 200, "max_temp": 220,
                  "flights": 12, "positions_per_flight": 30}


def dataset_templates() -> dict:
    out = {}
    for d in sorted(os.listdir(DATASET_DIR)):
        p = os.path.join(DATASET_DIR, d, "dataset.json")
        if os.path.exists(p):
            with open(p) as f:
                meta = json.load(f)
            out[meta["id"]] = meta
    return out


def params() -> dict:
    out = {}
    for k, v in PARAM_DEFAULTS.items():
        env = os.environ.get("SITEWHERE_DATASET_" + k.upper())
        out[k] = type(v)(env) if env is not None else v
    return out


class _Geo:
    """Geometry helpers for initializer scripts (scripts cannot import numpy)."""

    @staticmethod
    def contains(bounds, lat: float, lon: float) -> bool:
        from ..core.geo import contains, polygon_of
        return bool(contains(polygon_of(bounds), lat, lon))

    @staticmethod
    def centroid(bounds) -> tuple[float, float]:
        pts = [(b["latitude"], b["longitude"]) if isinstance(b, dict) else (b.latitude, b.longitude) for b in bounds]
        return sum(p[0] for p in pts) / len(pts), sum(p[1] for p in pts) / len(pts)


def _source(engine, script: str, path: str) -> str:
    """The tenant's active override of ``script`` if one is stored, else the packaged file."""
    sid = "initializer-" + os.path.splitext(os.path.basename(script))[0]
    scripts = getattr(engine.ms.instance, "scripts", None)
    if scripts is not None:
        try:
            return scripts.get_content(engine.tenant.token, engine.ms.identifier, sid)
        except Exception:  # noqa: BLE001 -- no override stored
            pass
    with open(path) as f:
        return f.read()


def run_initializers(engine, section: str, template: str | None, bindings: dict, seed: int = 7) -> int:
    """Run the ``section`` initializers of dataset ``template`` for ``engine``'s tenant; returns how
    many scripts ran."""
    from ..runtime.scripting import _SAFE_BUILTINS, _restricted_import, check_source
    if not template or template == "empty":
        return 0
    meta = dataset_templates().get(template)
    if meta is None:
        raise ValueError(f"unknown dataset template {template!r}")
    log = logging.getLogger(f"sitewhere.dataset.{template}")
    ran = 0
    for script in meta.get("initializers", {}).get(section, []):
        path = os.path.join(DATASET_DIR, template, script)
        ns = {"__builtins__": dict(_SAFE_BUILTINS, __import__=_restricted_import), "__name__": f"initializer:{script}",
              "logger": log, "rnd": random.Random(seed), "params": params(), "geo": _Geo(), **bindings}
        src = _source(engine, script, path)
        check_source(src, path)
        exec(compile(src, path, "exec"), ns)  # noqa: S102 -- restricted builtins, checked source
        ran += 1
    return ran
