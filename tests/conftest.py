import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    # durable tenant stores (segments) of this test process go to a fresh directory
    if "SITEWHERE_DATA_DIR" not in os.environ:
        import tempfile
        os.environ["SITEWHERE_DATA_DIR"] = tempfile.mkdtemp(prefix="sw-test-data-")
    # dataset initializers (sitewhere_amd/datasets) build small tenants under test
    for k, v in (("DEVICES_PER_SITE", "3"), ("MEASUREMENTS_PER_ASSIGNMENT", "10"), ("LOCATIONS_PER_ASSIGNMENT", "8"),
                 ("FLIGHTS", "4"), ("POSITIONS_PER_FLIGHT", "6")):
        os.environ.setdefault("SITEWHERE_DATASET_" + k, v)
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def engine_knows(ib, dev) -> bool:
    """An inbound tenant engine has ``dev`` and its active assignment in the engine's own tables.
    Its index entries are taken before the engine update they key (under the engine lock), so
    waiting on the index alone races the first batch, which then routes the device as unregistered."""
    di, ai = ib.dev_index.idx.get(dev.id), ib.asg_index.idx.get(dev.device_assignment_id)
    if di is None or ai is None:
        return False
    from sitewhere_amd.pipeline.fleet import fingerprint_str
    with ib._lock:
        # the device's fingerprint too: an assignment's update can precede its device's
        return (int(ib.engine.dev_asg[di]) == ai and bool(ib.engine.asg_active[ai])
                and ib.engine.lookup_device(*fingerprint_str(dev.token)) == di)


@pytest.fixture(autouse=True)
def _fresh_data_dir(tmp_path_factory, monkeypatch):
    """Each test's durable tenant stores (``${sitewhere.data.dir}``) start empty: tests reuse tenant
    tokens across instances, and a store reopened from an earlier test would hold its events."""
    monkeypatch.setenv("SITEWHERE_DATA_DIR", str(tmp_path_factory.mktemp("sw-data")))


@pytest.fixture(scope="session")
def native_lib():
    from sitewhere_amd._native import native
    return native()
