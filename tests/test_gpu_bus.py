"""MI355X engine on commit-log topics without host copies (pipeline/bus_io.py).

Raw batches are published to a topic as pinned zero-copy records, read in place and DMA'd to HBM;
enriched rows are DMA'd by the copy engine into pinned records published to the enriched-batch
topic.  Every row must match the CPU oracle, a plain reader of the topic must see the same rows,
and retention must hand the row buffers back to the publisher's pool."""
import numpy as np
import pytest

from tests.conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs an MI355X GPU")]

from sitewhere_amd.bus.log import EventBus
from sitewhere_amd.pipeline.cpu_engine import CpuInboundEngine
from sitewhere_amd.pipeline.framing import varint_lengths

from pipeline_scenarios import NOW, setup_fleet, small_cfg, fleet_batch, canon_out


def test_engine_consumes_and_publishes_topics_in_place():
    from sitewhere_amd.pipeline.bus_io import OutboundPublisher, RawBatchRecord, raw_view, read_out_batch
    from sitewhere_amd.pipeline.gpu_engine import GpuInboundEngine, PipelinedRunner
    g, c = GpuInboundEngine(small_cfg()), CpuInboundEngine(small_cfg())
    setup_fleet(g, n_dev=1000)
    setup_fleet(c, n_dev=1000)
    bus = EventBus(default_partitions=1)
    bus.topic("raw", 1)
    pub = OutboundPublisher(bus, "enriched", g.lib, g.out_cap, retention_bytes=250_000)   # ~2 batches of rows
    runner = PipelinedRunner(g, max_raw_bytes=1 << 20, out_target=pub.target, on_outbound=pub.publish)
    reader = bus.consumer("downstream", ["enriched"])
    cpu_rows, seen = [], []
    for k in range(8):
        raw, offs = fleet_batch(2000, seed=900 + k)
        rec = RawBatchRecord(raw[:int(offs[-1])], varint_lengths(offs), len(offs) - 1)
        off = rec.publish(bus, "raw", ts=NOW + k)
        payload, lens, n, pb = raw_view(bus.view("raw", 0, off))
        assert payload.is_pinned() and n == len(offs) - 1 and pb == int(offs[-1])
        assert payload.data_ptr() == rec.ptr + 64         # read in place, not copied
        runner.submit(payload, None, n, now_ms=NOW + k, lens_host=lens, raw_bytes=pb)
        r = c.step(raw, offs, NOW + k, presence=False)
        cpu_rows.append(r.out)
        for recs in reader.poll(0).values():                                  # a lagging reader keeps up
            seen += [read_out_batch(x.value)[1].copy() for x in recs]
    runner.flush()
    for recs in reader.poll(200).values():
        seen += [read_out_batch(x.value)[1].copy() for x in recs]
    assert pub.published == 8 and len(seen) == 8
    assert g.stats_dict() == c.stats_dict()
    assert canon_out(np.concatenate(seen), None) == canon_out(np.concatenate(cpu_rows), None)
    assert pub.rows == sum(len(x) for x in cpu_rows)
    assert pub.n_alloc < 8                 # retention returned row buffers to the pool and they were reused
