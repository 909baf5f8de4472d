"""Engine-shard checkpoint / resume: a restored shard replays the batches after the
snapshot to exactly the outputs, event ids, device state and statistics of the uninterrupted run."""
import numpy as np
import pytest

from sitewhere_amd.pipeline.checkpoint import read_meta
from sitewhere_amd.pipeline.cpu_engine import CpuInboundEngine

from pipeline_scenarios import NOW, setup_fleet, small_cfg, fleet_batch, canon_out, SQUARE
from tests.conftest import gpu_available


def _zones(e):
    from sitewhere_amd.pipeline.engine_base import Zone, ZoneTest
    e.set_zone_rules([Zone("z1", SQUARE)], [ZoneTest("z1", "inside", "zone.enter", 2, "entered")])


def _run(e, batches, t0):
    out = []
    for k, (raw, offs) in enumerate(batches):
        r = e.step(raw, offs, t0 + k * 1000, presence=(k == len(batches) - 1))
        out.append((r.n_events, r.n_persisted, canon_out(r.out, None), r.event_ids().tolist(),
                    sorted(zip(r.reject_status.tolist(), [bytes(x) for x in r.rejects.view(np.uint8)]))))
    return out


def _roundtrip(make, tmp_path, include_store=False):
    batches = [fleet_batch(1500, seed=900 + k) for k in range(6)]
    a = make()
    setup_fleet(a)
    _zones(a)
    _run(a, batches[:3], NOW)
    path = str(tmp_path / "shard.safetensors")
    a.save_checkpoint(path, include_store=include_store, extra={"offsets": {"raw-0": 42}})
    tail_a = _run(a, batches[3:], NOW + 10_000_000)     # late enough that presence fires
    b = make()
    extra = b.load_checkpoint(path)
    assert extra == {"offsets": {"raw-0": 42}}
    tail_b = _run(b, batches[3:], NOW + 10_000_000)
    assert tail_a == tail_b
    assert a.stats_dict() == b.stats_dict()
    for asg in (0, 1, 7, 123):
        assert a.device_state(asg) == b.device_state(asg)
    return a, b, path


def test_cpu_checkpoint_resume_is_exact(tmp_path):
    _, _, path = _roundtrip(lambda: CpuInboundEngine(small_cfg()), tmp_path, include_store=True)
    meta = read_meta(path)
    assert meta["kind"] == "cpu" and meta["n_devices"] == 1000


def test_checkpoint_rejects_other_sizing(tmp_path):
    a = CpuInboundEngine(small_cfg())
    setup_fleet(a)
    path = str(tmp_path / "x.safetensors")
    a.save_checkpoint(path)
    with pytest.raises(ValueError, match="sizing"):
        CpuInboundEngine(small_cfg(max_devices=8192)).load_checkpoint(path)


def test_cpu_checkpoint_keeps_shuffle_carry(tmp_path):
    """A shard whose full slabs deferred records resumes with the same carry."""
    from sitewhere_amd.pipeline.config import EngineConfig
    cfg = dict(world=3, rank=1, shuffle_slack=0.1, shuffle_pad=0)
    a = CpuInboundEngine(EngineConfig.small(**cfg))
    setup_fleet(a)
    recs, _ = a.decode_phase(*fleet_batch(3000, seed=5), NOW)
    a.partition(recs)
    assert len(a.carry) > 0
    path = str(tmp_path / "c.safetensors")
    a.save_checkpoint(path)
    b = CpuInboundEngine(EngineConfig.small(**cfg))
    b.load_checkpoint(path)
    assert b.carry.tobytes() == a.carry.tobytes()


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs an MI355X GPU")
def test_gpu_checkpoint_resume_is_exact(tmp_path):
    from sitewhere_amd.pipeline.gpu_engine import GpuInboundEngine
    a, b, path = _roundtrip(lambda: GpuInboundEngine(small_cfg()), tmp_path)
    with pytest.raises(ValueError, match="cannot restore"):
        CpuInboundEngine(small_cfg()).load_checkpoint(path)
