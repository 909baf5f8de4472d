"""Native multi-threaded CPU engine (csrc/native/swcpuengine.cpp) against the Python oracle.

Every observable must match bit for bit: outbound rows (order included), reject rows and statuses,
the event-store ring, device state (last location / measurement / alert per assignment), interned
names, stats, and checkpoint/resume.  Covers 1 and several worker threads (sharded dedup and
state merge), zone rules, presence, duplicates within and across batches and store wraparound.
"""
import numpy as np
import pytest

from sitewhere_amd.pipeline.cpu_engine import CpuInboundEngine
from sitewhere_amd.pipeline.native_engine import NativeCpuEngine

from pipeline_scenarios import NOW, fleet_batch, hand_batch, setup_fleet, small_cfg


def pair(threads, **cfg):
    o = CpuInboundEngine(small_cfg(**cfg))
    n = NativeCpuEngine(small_cfg(**cfg), threads=threads)
    for e in (o, n):
        setup_fleet(e, n_dev=300)
    return o, n


def same_result(ro, rn):
    assert ro.n_events == rn.n_events and ro.n_persisted == rn.n_persisted
    assert ro.first_seq == rn.first_seq
    assert ro.out.tobytes() == rn.out.tobytes()
    assert ro.rejects.tobytes() == rn.rejects.tobytes()
    assert np.array_equal(ro.reject_status, rn.reject_status)
    assert ro.new_names == rn.new_names


def same_engine(o, n):
    assert o.stats_dict() == n.stats_dict()
    assert o.cursor == n.cursor and o.seq_base == n.seq_base
    assert o.intern == n.intern_table()
    co, eo = o.store_rows()
    cn, en = n.store_rows()
    assert np.array_equal(eo, en)
    for k in co:
        assert np.array_equal(co[k], cn[k]), k
    for k in ("st_last", "st_missing", "st_loc_date", "st_loc_eid"):
        assert np.array_equal(getattr(o, k), getattr(n, k)), k
    for a in range(o.n_assignments):
        assert o.device_state(a) == n.device_state(a)


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_hand_batch_matches_oracle(threads):
    o, n = pair(threads)
    raw, offs = hand_batch()
    for k in range(3):                       # repeats: cross-batch duplicates
        same_result(o.step(raw, offs, NOW + k, presence=False), n.step(raw, offs, NOW + k, presence=False))
    same_engine(o, n)


@pytest.mark.parametrize("threads", [1, 4])
def test_fleet_multi_step_with_presence_and_wraparound(threads):
    # store_cap small enough that the ring wraps during the run
    o, n = pair(threads, store_cap=1 << 13)
    for step in range(6):
        raw, offs = fleet_batch(1500, seed=100 + step % 4, n_dev=300)   # seeds repeat -> duplicates
        now = NOW + step * 1000
        same_result(o.step(raw, offs, now, presence=False), n.step(raw, offs, now, presence=False))
    later = NOW + o.cfg.presence_missing_ms + 10_000
    empty = (np.zeros(64, np.uint8), np.zeros(1, np.uint32))
    same_result(o.step(*empty, later, presence=True), n.step(*empty, later, presence=True))
    same_result(o.step(*empty, later + 5, presence=True), n.step(*empty, later + 5, presence=True))
    same_engine(o, n)


def test_gen_cap_truncates_like_oracle():
    o, n = pair(4, gen_cap=16)
    raw, offs = fleet_batch(2000, seed=5, n_dev=300)
    same_result(o.step(raw, offs, NOW, presence=False), n.step(raw, offs, NOW, presence=False))
    same_engine(o, n)


def test_checkpoint_resume_continues_identically(tmp_path):
    o, n = pair(4)
    raw, offs = fleet_batch(1200, seed=9, n_dev=300)
    o.step(raw, offs, NOW, presence=False)
    n.step(raw, offs, NOW, presence=False)
    path = str(tmp_path / "shard.safetensors")
    n.save_checkpoint(path, include_store=True)
    n2 = NativeCpuEngine(small_cfg(), threads=2)      # different thread count: state re-shards
    setup_fleet(n2, n_dev=300)
    n2.load_checkpoint(path)
    raw2, offs2 = fleet_batch(1200, seed=9, n_dev=300)  # same alternate ids -> all duplicates
    same_result(o.step(raw2, offs2, NOW + 1, presence=False), n2.step(raw2, offs2, NOW + 1, presence=False))
    same_engine(o, n2)


def test_oracle_checkpoint_loads_into_native(tmp_path):
    o, _ = pair(1)
    raw, offs = fleet_batch(800, seed=3, n_dev=300)
    o.step(raw, offs, NOW, presence=False)
    path = str(tmp_path / "oracle.safetensors")
    o.save_checkpoint(path, include_store=True)
    n = NativeCpuEngine(small_cfg(), threads=4)
    setup_fleet(n, n_dev=300)
    n.load_checkpoint(path)
    same_engine(o, n)
