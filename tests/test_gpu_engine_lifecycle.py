"""GPU engines created one after another in one process (the caching allocator hands each the HBM
its predecessors freed), with devices registered from a second thread while the first thread steps
batches, as a tenant's model-update feed does: a batch from a registered device persists in full."""
from __future__ import annotations

import pytest


@pytest.mark.gpu
@pytest.mark.skipif(not __import__("conftest").gpu_available(), reason="needs an MI355X GPU")
def test_engines_back_to_back_register_from_another_thread():
    import scripts.engine_reuse_probe as probe
    for k in range(4):
        cap = probe.COLUMNAR if k % 2 == 0 else {}
        r = probe.one(k, cap, threaded=k < 2, encode=True)
        assert r["persisted"] == r["expected"], r
        assert r["step_counters"].get("unregistered") == 1, r
