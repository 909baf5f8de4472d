"""Raw-batch framing: payload bytes + one LEB128 varint length per payload.

The MI355X pipeline is bound by the H2D copy of each raw batch (PCIe, ~56 GB/s measured).  u32
offsets cost 4 B per payload on that link; a varint length costs 1 B for payloads under 128 B
(the reference's protobuf device messages are ~50-60 B), and the GPU rebuilds the offsets with a
scan (``sw_frame_varint`` in ``csrc/hip/swgpu.hip``).  Kafka record batches frame records with the
same zig-zag-free varints (reference event sources hand each payload to Kafka as one record,
``EventSourcesMicroservice`` -> ``DecodedEventsProducer``).
"""
from __future__ import annotations

import numpy as np


def varint_lengths(offs: np.ndarray) -> np.ndarray:
    """u32/i64 offsets (n + 1) -> LEB128 length stream (uint8)."""
    lens = np.diff(np.asarray(offs, np.int64))
    if len(lens) and lens.min() < 0:
        raise ValueError("offsets must be non-decreasing")
    nb = 1 + sum((lens >= (1 << (7 * k))).astype(np.int64) for k in range(1, 5))
    out = np.empty(int(nb.sum()), np.uint8)
    pos = np.zeros(len(lens), np.int64)
    if len(lens) > 1:
        np.cumsum(nb[:-1], out=pos[1:])
    for k in range(5):
        sel = nb > k
        if not sel.any():
            break
        group = (lens[sel] >> (7 * k)) & 0x7F
        cont = (nb[sel] > k + 1).astype(np.int64) << 7
        out[pos[sel] + k] = (group | cont).astype(np.uint8)
    return out


def offsets_from_varint(stream: np.ndarray) -> np.ndarray:
    """Inverse of :func:`varint_lengths` (CPU reference of the GPU framing kernels)."""
    b = np.asarray(stream, np.uint8)
    lens, v, shift = [], 0, 0
    for x in b.tolist():
        v |= (x & 0x7F) << shift
        if x & 0x80:
            shift += 7
        else:
            lens.append(v)
            v, shift = 0, 0
    offs = np.zeros(len(lens) + 1, np.int64)
    np.cumsum(lens, out=offs[1:])
    return offs.astype(np.uint32)
