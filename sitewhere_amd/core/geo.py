"""Geospatial helpers (reference ``sitewhere-core/.../geospatial/GeoUtils.java:26-65`` over JTS).

Point-in-polygon uses the even-odd crossing test (the same predicate as the gfx950 ``pip``
kernel); ``batch_contains`` dispatches large batches to ``libswgpu`` when a GPU is present.
"""
from __future__ import annotations

import math

import numpy as np


def polygon_of(bounds) -> np.ndarray:
    """Zone/area bounds (list of Location or dicts) -> (N, 2) float64 [lat, lon]."""
    pts = []
    for b in bounds:
        if isinstance(b, dict):
            pts.append((float(b["latitude"]), float(b["longitude"])))
        elif hasattr(b, "latitude"):
            pts.append((float(b.latitude), float(b.longitude)))
        else:
            pts.append((float(b[0]), float(b[1])))
    return np.asarray(pts, np.float64).reshape(-1, 2)


def contains(poly: np.ndarray, lat: float, lon: float) -> bool:
    inside = False
    n = len(poly)
    j = n - 1
    for i in range(n):
        xi, yi = poly[i]
        xj, yj = poly[j]
        if ((yi > lon) != (yj > lon)) and (lat < (xj - xi) * (lon - yi) / (yj - yi) + xi):
            inside = not inside
        j = i
    return inside


def batch_contains(polys: list[np.ndarray], pts: np.ndarray, use_gpu: bool | None = None) -> np.ndarray:
    """[P points x Z zones] containment matrix; GPU kernel ``sw_pip_batch`` for big batches."""
    pts = np.ascontiguousarray(pts, np.float64).reshape(-1, 2)
    if use_gpu is None:
        use_gpu = len(pts) * len(polys) >= 1 << 16 and _gpu_ok()
    if use_gpu:
        import ctypes
        import torch
        from .._native import gpu
        off = np.zeros(len(polys) + 1, np.int32)
        off[1:] = np.cumsum([len(p) for p in polys])
        vtx = np.concatenate([p.ravel() for p in polys]) if polys else np.zeros(2)
        d = torch.device("cuda")
        out = torch.zeros(len(pts) * len(polys), dtype=torch.uint8, device=d)
        pt, vt, ot = (torch.from_numpy(x).to(d) for x in (pts.ravel().copy(), vtx, off))
        rc = gpu().sw_pip_batch(pt.data_ptr(), len(pts), vt.data_ptr(), ot.data_ptr(), len(polys), out.data_ptr(),
                                ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        if rc:
            raise RuntimeError(f"sw_pip_batch failed ({rc})")
        return out.cpu().numpy().reshape(len(pts), len(polys)).astype(bool)
    res = np.zeros((len(pts), len(polys)), bool)
    for z, poly in enumerate(polys):
        for p, (la, lo) in enumerate(pts):
            res[p, z] = contains(poly, la, lo)
    return res


def _gpu_ok() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def haversine_m(lat1, lon1, lat2, lon2) -> float:
    r = 6371000.0
    p1, p2 = math.radians(lat1), math.radians(lat2)
    dp, dl = p2 - p1, math.radians(lon2 - lon1)
    a = math.sin(dp / 2) ** 2 + math.cos(p1) * math.cos(p2) * math.sin(dl / 2) ** 2
    return 2 * r * math.asin(math.sqrt(a))
