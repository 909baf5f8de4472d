"""gfx950 decode kernels vs an independent decoder (``tests/decode_oracle.py``), bitwise.

The host engine compiles the same ``swdecode.h`` as the kernels, so GPU-vs-host parity alone only
shows both compilers agree; here the device records are checked against a pure-Python decoder
written from the protobuf wire rules and the reference schema, on generator batches, hand-built
edge cases and random corruptions (truncations, flips, insertions, garbage), across the LDS-staged
and the direct-from-HBM paths of ``k_decode_count`` / ``k_decode_emit``.
"""
import numpy as np
import pytest

from tests.conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs an MI355X GPU")]

if gpu_available():
    from sitewhere_amd.pipeline.gpu_engine import GpuInboundEngine

from decode_oracle import decode_batch
from pipeline_scenarios import small_cfg
from test_decode import NOW, oracle_batch


def test_device_decode_matches_independent_oracle_bitwise():
    raw, offs = oracle_batch(seed=23)
    want, why = decode_batch(raw, offs, NOW)
    g = GpuInboundEngine(small_cfg(max_msgs=8192, rec_cap=len(want) + 1024))
    got = g.decode_only(raw, offs, NOW)
    assert len(got) == len(want)
    bad = np.nonzero((got.view(np.uint8).reshape(-1, 80) != want.view(np.uint8).reshape(-1, 80)).any(1))[0]
    assert bad.size == 0, (bad[:5], got[bad[:3]], want[bad[:3]])
    assert sum(w is not None for w in why) > 1000


def test_device_decode_of_corrupted_batches_never_escapes_its_payload():
    """Every record of a garbage-heavy batch points inside its own payload (no out-of-range aux
    offsets for the host to follow) and matches the oracle."""
    from decode_oracle import mutated_payloads
    from sitewhere_amd.pipeline.fleet import pack_messages
    msgs = mutated_payloads(99, 6000, NOW)
    raw, offs = pack_messages(msgs)
    want, _ = decode_batch(raw, offs, NOW)
    g = GpuInboundEngine(small_cfg(max_msgs=8192, rec_cap=len(want) + 1024))
    got = g.decode_only(raw, offs, NOW)
    assert np.array_equal(got.view(np.uint8), want.view(np.uint8))
    end = int(offs[-1])
    assert (got["aux_off"].astype(np.int64) + got["aux_len"] <= end).all()
    assert (got["aux2_off"].astype(np.int64) + got["aux2_len"] <= end).all()


def test_device_string_refs_match_independent_oracle():
    """The string refs k_decode_emit writes beside each record (alternate id, metadata span,
    measurement index -- the durable record's strings) equal the oracle's, and oversize events are
    one host-routed record, as on the host."""
    from sitewhere_amd.models import wire
    from sitewhere_amd.pipeline.fleet import pack_messages
    raw, offs = oracle_batch(seed=29)
    b = raw[:int(offs[-1])].tobytes()
    msgs = [b[offs[i]:offs[i + 1]] for i in range(len(offs) - 1)]
    msgs += [wire.alert("d-1", "t", "x" * 70000), wire.measurements("d-2", {"a": 1.0}, alternate_id="y" * 66000)]
    raw, offs = pack_messages(msgs)
    want, why, wsp = decode_batch(raw, offs, NOW, spans=True)
    g = GpuInboundEngine(small_cfg(max_msgs=16384, rec_cap=len(want) + 1024))
    got, gsp = g.decode_only(raw, offs, NOW, spans=True)
    assert np.array_equal(got.view(np.uint8), want.view(np.uint8))
    assert np.array_equal(gsp.view(np.uint8), wsp.view(np.uint8))
    assert why[-2:] == ["oversize", "oversize"] and (gsp["has"] & 2).sum() > 50
