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
    """Inverse of :func:`varint_lengths` (CPU reference of the GPU framing kernels), vectorised:
    a byte without the continuation bit ends a length; each byte contributes its low 7 bits shifted
    by 7 x its position inside its length."""
    b = np.asarray(stream, np.uint8)
    end = (b & 0x80) == 0
    if len(b) and not end[-1]:
        raise ValueError("truncated varint length stream")
    n = int(end.sum())
    offs = np.zeros(n + 1, np.int64)
    if n:
        grp = np.zeros(len(b), np.int64)
        np.cumsum(end[:-1], out=grp[1:])                   # length index of every byte
        first = np.zeros(n, np.int64)
        first[1:] = np.nonzero(end)[0][:-1] + 1            # first byte of every length
        shift = 7 * (np.arange(len(b), dtype=np.int64) - first[grp])
        if len(shift) and int(shift.max()) > 28:           # > 5 bytes: not a u32 length
            raise ValueError("over-long varint length")
        vals = (b & 0x7F).astype(np.int64) << shift
        np.cumsum(np.bincount(grp, weights=vals, minlength=n).astype(np.int64), out=offs[1:])
    return offs.astype(np.uint32)
