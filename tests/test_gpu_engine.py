"""GPU engine (libswgpu.so on gfx950) vs the CPU oracle engine -- bitwise parity where deterministic.

Validated events persist in stable order on both engines, so their event ids, store rows and
outbound rows match exactly; generated rule/presence events are compared as multisets.
"""
import numpy as np
import pytest

from tests.conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs an MI355X GPU")]

if gpu_available():
    import torch
    from sitewhere_amd.pipeline.gpu_engine import GpuInboundEngine, PipelinedRunner

from sitewhere_amd.models.columnar import EV_STATE_CHANGE
from sitewhere_amd.pipeline.cpu_engine import CpuInboundEngine

from pipeline_scenarios import NOW, setup_fleet, small_cfg, hand_batch, fleet_batch, canon_out


def pair(**kw):
    g = GpuInboundEngine(small_cfg(**kw))
    c = CpuInboundEngine(small_cfg(**kw))
    setup_fleet(g, n_dev=1000)
    setup_fleet(c, n_dev=1000)
    return g, c


def assert_same_step(rg, rc, names):
    assert rg.n_events == rc.n_events
    assert rg.n_persisted == rc.n_persisted
    assert canon_out(rg.out, names) == canon_out(rc.out, names)
    # rejected records: same multiset of (status, bytes)
    kg = sorted(zip(rg.reject_status.tolist(), [bytes(x) for x in rg.rejects.view(np.uint8).reshape(-1, 80)]))
    kc = sorted(zip(rc.reject_status.tolist(), [bytes(x) for x in rc.rejects.view(np.uint8).reshape(-1, 80)]))
    assert kg == kc


def test_abi_sizes_match():
    from sitewhere_amd._native import gpu
    from sitewhere_amd.ops.engine_abi import abi_sizes, SwEngineArgs
    import ctypes
    s = abi_sizes(gpu())
    assert s["event_rec"] == 80 and s["out_rec"] == 32 and s["name_ref"] == 16
    assert s["engine_args"] == ctypes.sizeof(SwEngineArgs)
    assert [s["reg_slot"], s["asg_state"], s["ms_slot"]] == [32, 32, 32]
    from sitewhere_amd.models.columnar import WIRE_REC
    assert s["wire_rec"] == WIRE_REC.itemsize == 64


def test_hand_batch_parity():
    g, c = pair()
    raw, offs = hand_batch()
    rg = g.step(raw, offs, NOW, presence=False)
    rc = c.step(raw, offs, NOW, presence=False)
    assert_same_step(rg, rc, c.names)
    assert g.stats_dict() == c.stats_dict()
    assert rg.new_names == rc.new_names


def test_fleet_parity_multi_step_with_state():
    g, c = pair()
    for k in range(4):
        raw, offs = fleet_batch(3000, seed=100 + k)
        rg = g.step(raw, offs, NOW + k * 1000, presence=False)
        rc = c.step(raw, offs, NOW + k * 1000, presence=False)
        assert_same_step(rg, rc, c.names)
    assert g.stats_dict() == c.stats_dict()
    # store contents (ordered part: everything but generated rows)
    cg, eg = g.store_rows()
    cc, ec = c.store_rows()
    assert np.array_equal(eg, ec)
    for k in ("etype", "dev", "asg", "cust", "area", "asset", "date", "recv"):
        assert sorted(cg[k].tolist()) == sorted(cc[k].tolist()), k
    # device state for a sample of assignments
    for a in range(0, 1000, 37):
        sg, sc = g.device_state(a), c.device_state(a)
        assert sg["last_interaction"] == sc["last_interaction"]
        assert sg["measurements"].keys() == sc["measurements"].keys()
        for name in sc["measurements"]:
            assert sg["measurements"][name][1] == sc["measurements"][name][1]
        if sc["last_location"]:
            assert sg["last_location"][1] == sc["last_location"][1]


def test_presence_parity():
    g, c = pair()
    raw, offs = fleet_batch(2000, seed=5)
    g.step(raw, offs, NOW, presence=False)
    c.step(raw, offs, NOW, presence=False)
    later = NOW + g.cfg.presence_missing_ms + 5
    empty_raw, empty_off = np.zeros(64, np.uint8), np.zeros(1, np.uint32)
    rg = g.step(empty_raw, empty_off, later, presence=True)
    rc = c.step(empty_raw, empty_off, later, presence=True)
    assert (rg.out["etype"] == EV_STATE_CHANGE).sum() == (rc.out["etype"] == EV_STATE_CHANGE).sum() > 0
    assert sorted(rg.out["assignment"].tolist()) == sorted(rc.out["assignment"].tolist())


@pytest.mark.parametrize("mode", ["direct", "push", "sdma", "hsa"])
def test_pipelined_runner_matches_sync(mode):
    g, c = pair()
    seen = []
    runner = PipelinedRunner(g, max_raw_bytes=1 << 20, on_outbound=lambda rows: seen.append(rows.copy()), mode=mode)
    batches = [fleet_batch(2000, seed=300 + k) for k in range(5)]
    total = 0
    cpu_rows = []
    for k, (raw, offs) in enumerate(batches):
        rh = torch.from_numpy(raw).pin_memory()
        oh = torch.from_numpy(offs.view(np.int32)).pin_memory()
        runner.submit(rh, oh, len(offs) - 1, now_ms=NOW + k)
        r = c.step(raw, offs, NOW + k, presence=False)
        total += r.n_persisted
        cpu_rows.append(r.out)
    runner.flush()
    assert runner.delivered == total == sum(len(x) for x in seen)
    assert g.stats_dict() == c.stats_dict()
    assert canon_out(np.concatenate(seen), None) == canon_out(np.concatenate(cpu_rows), None)


def test_varint_framing_kernel_matches_host_offsets():
    from sitewhere_amd.pipeline.framing import varint_lengths
    g = GpuInboundEngine(small_cfg(max_msgs=8192))
    rng = np.random.default_rng(5)
    lens = np.concatenate([rng.integers(0, 128, 5000), rng.integers(128, 70000, 200), [0, 127, 128, 16383, 16384]])
    rng.shuffle(lens)
    offs = np.zeros(len(lens) + 1, np.int64)
    np.cumsum(lens, out=offs[1:])
    stream = varint_lengths(offs)
    assert len(stream) > len(lens)              # some multi-byte varints cross tile boundaries
    ld = torch.from_numpy(stream).cuda()
    od = torch.full((len(lens) + 8,), -1, dtype=torch.int32, device="cuda")
    g.frame_varint(ld, len(stream), len(lens), od, int(offs[-1]))
    torch.cuda.synchronize()
    assert np.array_equal(od[:len(lens) + 1].cpu().numpy().view(np.uint32).astype(np.int64), offs)


def test_pipelined_runner_varint_framing_matches_sync():
    from sitewhere_amd.pipeline.framing import varint_lengths
    g, c = pair()
    seen = []
    runner = PipelinedRunner(g, max_raw_bytes=1 << 20, on_outbound=lambda rows: seen.append(rows.copy()))
    total = 0
    cpu_rows = []
    for k in range(4):
        raw, offs = fleet_batch(2000, seed=700 + k)
        rh = torch.from_numpy(raw).pin_memory()
        lh = torch.from_numpy(varint_lengths(offs)).pin_memory()
        runner.submit(rh, None, len(offs) - 1, now_ms=NOW + k, lens_host=lh, raw_bytes=int(offs[-1]))
        r = c.step(raw, offs, NOW + k, presence=False)
        total += r.n_persisted
        cpu_rows.append(r.out)
    runner.flush()
    assert runner.delivered == total == sum(len(x) for x in seen)
    assert g.stats_dict() == c.stats_dict()
    assert canon_out(np.concatenate(seen), None) == canon_out(np.concatenate(cpu_rows), None)


def test_standalone_pip_kernel():
    import ctypes
    from sitewhere_amd._native import gpu
    from sitewhere_amd.pipeline.cpu_engine import pip
    rng = np.random.default_rng(0)
    poly = np.array([(0, 0), (0, 4), (2, 2), (4, 4), (4, 0)], np.float64)
    pts = rng.uniform(-1, 5, size=(4096, 2))
    d = torch.device("cuda")
    out = torch.zeros(len(pts), dtype=torch.uint8, device=d)
    vt = torch.from_numpy(poly.ravel()).to(d)
    off = torch.tensor([0, len(poly)], dtype=torch.int32, device=d)
    pt = torch.from_numpy(pts.ravel()).to(d)
    rc = gpu().sw_pip_batch(pt.data_ptr(), len(pts), vt.data_ptr(), off.data_ptr(), 1, out.data_ptr(),
                            ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0
    got = out.cpu().numpy().astype(bool)
    want = np.array([pip(poly, x, y) for x, y in pts])
    assert (got == want).all()


def test_graph_replay_matches_direct_launches_and_recaptures_on_zone_change():
    """The hipGraph-captured process phase gives the same results as direct launches, including
    across a zone-rule change (which must re-capture: zone pointers are by-value kernel args)."""
    from sitewhere_amd.pipeline.engine_base import Zone, ZoneTest
    g = GpuInboundEngine(small_cfg())
    d = GpuInboundEngine(small_cfg())
    d.use_graph = False
    for e in (g, d):
        setup_fleet(e, n_dev=1000)
    for k in range(6):
        if k == 3:
            for e in (g, d):
                e.set_zone_rules([Zone("z2", [(32.0, -86.0), (32.0, -84.0), (34.5, -84.0), (34.5, -86.0)])],
                                 [ZoneTest("z2", "inside", "zone2.enter", 3)])
        raw, offs = fleet_batch(2500, seed=700 + k)
        rg = g.step(raw, offs, NOW + k * 1000, presence=(k == 5))
        rd = d.step(raw, offs, NOW + k * 1000, presence=(k == 5))
        assert canon_out(rg.out, None) == canon_out(rd.out, None)
        assert g.stats_dict() == d.stats_dict()
    assert g._graph is not None


def test_store_ring_wraparound_parity():
    """The HBM event ring wraps (store_cap << events): GPU ring contents and ids match the oracle."""
    g, c = pair(store_cap=4096)
    for k in range(5):
        raw, offs = fleet_batch(1500, seed=900 + k)
        rg = g.step(raw, offs, NOW + k * 1000, presence=False)
        rc = c.step(raw, offs, NOW + k * 1000, presence=False)
        assert rg.first_seq == rc.first_seq
        assert canon_out(rg.out, None) == canon_out(rc.out, None)
    assert g.cursor == c.cursor > 4096
    cg, eg = g.store_rows()
    cc, ec = c.store_rows()
    assert len(eg) == 4096 and np.array_equal(eg, ec)
    for k in ("etype", "asg", "date"):
        assert sorted(cg[k].tolist()) == sorted(cc[k].tolist()), k


@pytest.mark.gpu
def test_hot_store_query_kernel_matches_cpu_oracle():
    """k_store_filter + device ordering vs the CPU oracle's query_store after the HBM ring wrapped."""
    from sitewhere_amd.models.columnar import EV_ALERT, EV_LOCATION, EV_MEASUREMENT
    g = GpuInboundEngine(small_cfg(store_cap=1 << 12), device="cuda:0")
    c = CpuInboundEngine(small_cfg(store_cap=1 << 12))
    for e in (g, c):
        setup_fleet(e, n_dev=200)
    for k in range(5):
        raw, offs = fleet_batch(1500, seed=70 + k, n_dev=200)
        g.step(raw, offs, NOW + k, presence=False)
        c.step(raw, offs, NOW + k, presence=False)
    assert g.cursor == c.cursor > g.cfg.store_cap
    for et, asg, lo, hi, pn, ps in ((EV_MEASUREMENT, [1, 2, 3, 150], None, None, 1, 10),
                                    (EV_LOCATION, list(range(0, 200, 3)), NOW - 40_000, NOW, 2, 25),
                                    (EV_ALERT, list(range(200)), None, None, 1, 0)):
        tg, pg, eg = g.query_store(et, asg, lo, hi, pn, ps)
        tc, pc, ec = c.query_store(et, asg, lo, hi, pn, ps)
        assert tg == tc and np.array_equal(eg, ec)
        for k in ("date", "asg", "v0", "v1", "etype"):
            assert np.array_equal(pg[k], pc[k]), k


def test_overlapped_framed_steps_match_sync_oracle():
    """submit_framed / drain_framed (the service tenant's overlapped steps): batch k is returned when
    batch k+2 is submitted, from pinned zero-copy records.  Every result -- rows, rejects, learned
    names, first store sequence -- equals the CPU oracle's synchronous step of the same batch, and a
    synchronous step is refused while a submission is pending."""
    from sitewhere_amd.pipeline.bus_io import RawBatchRecord, parse_raw_batch
    from sitewhere_amd.pipeline.framing import varint_lengths
    g, c = pair()
    recs, want, got = [], [], []
    for k in range(6):
        raw, offs = fleet_batch(2500, seed=700 + k)
        rec = RawBatchRecord(raw[:int(offs[-1])], varint_lengths(offs), len(offs) - 1)
        recs.append(rec)
        want.append(c.step(raw, offs, NOW + k, presence=False))
        got += g.submit_framed(parse_raw_batch(rec.buf.numpy()[:rec.value_len]), NOW + k, token=k, presence=False)
        assert [t for t, _ in got] == list(range(max(0, k - 1)))   # rows of k-1 are still copying
        assert g.framed_pending == min(k + 1, 2)
        if k == 2:
            with pytest.raises(RuntimeError, match="pending"):
                g.step(raw, offs, NOW, presence=False)
    got += g.drain_framed()
    assert [t for t, _ in got] == list(range(6)) and not g.framed_pending
    for (_, rg), rc in zip(got, want):
        assert_same_step(rg, rc, c.names)
        assert rg.first_seq == rc.first_seq and rg.new_names == rc.new_names
        assert rg.n_msgs == rc.n_msgs and rg.n_events == rc.n_events
    assert g.stats_dict() == c.stats_dict()
    assert sum(len(r.rejects) for _, r in got) > 0                # unregistered devices were rejected
