"""QR symbology (label generation) and schedule trigger math."""
from __future__ import annotations

import datetime as dt
import struct
import zlib

import pytest

from sitewhere_amd.models.domain import Schedule, TriggerType
from sitewhere_amd.services.qrcode import EC_TABLE, QrCode, decode_format_bits, gf_mul
from sitewhere_amd.services.schedule_management import CronExpression, next_fire


def _gf_pow2(i):
    x = 1
    for _ in range(i):
        x = gf_mul(x, 2)
    return x


def _poly_eval(cw, x):
    y = 0
    for c in cw:
        y = gf_mul(y, x) ^ c
    return y


def _read_back(q: QrCode) -> bytes:
    """Unmask, un-zigzag, de-interleave and parse the byte-mode segment."""
    n = q.size
    f = q._mask_fn(q.mask)
    bits = []
    right = n - 1
    while right >= 1:
        if right == 6:
            right = 5
        for vert in range(n):
            for j in range(2):
                x = right - j
                y = n - 1 - vert if ((right + 1) & 2) == 0 else vert
                if not q.function[y][x]:
                    bits.append(int(q.modules[y][x] ^ f(x, y)))
        right -= 2
    ecw, b1, d1, b2, d2 = EC_TABLE[q.ec][q.version - 1]
    total = b1 * d1 + b2 * d2 + ecw * (b1 + b2)
    cws = [int("".join(map(str, bits[i * 8:i * 8 + 8])), 2) for i in range(total)]
    sizes = [d1] * b1 + [d2] * b2
    blocks = [[] for _ in sizes]
    k = 0
    for i in range(max(sizes)):
        for b, s in enumerate(sizes):
            if i < s:
                blocks[b].append(cws[k])
                k += 1
    ecs = [[] for _ in sizes]
    for i in range(ecw):
        for b in range(len(sizes)):
            ecs[b].append(cws[k])
            k += 1
    for d, e in zip(blocks, ecs):   # every block is a valid RS codeword: zero syndromes
        assert all(_poly_eval(d + e, _gf_pow2(i)) == 0 for i in range(ecw))
    data = [b for blk in blocks for b in blk]
    bitstr = "".join(f"{b:08b}" for b in data)
    assert bitstr[:4] == "0100"
    cc = 8 if q.version < 10 else 16
    ln = int(bitstr[4:4 + cc], 2)
    start = 4 + cc
    return bytes(int(bitstr[start + 8 * i:start + 8 * i + 8], 2) for i in range(ln))


@pytest.mark.parametrize("text,ec", [("HELLO WORLD", "M"), ("sitewhere://default/device/galaxytab-000", "Q"),
                                     ("x" * 100, "L"), ("tenant-device-" * 8, "H"), ("ü-unicode ✓", "M")])
def test_qr_roundtrip(text, ec):
    q = QrCode(text, ec=ec)
    assert q.size == 17 + 4 * q.version
    assert _read_back(q) == text.encode()
    # format information decodes to (ec, mask) from both copies
    assert decode_format_bits(q.format_bits) == (ec, q.mask)
    n = q.size
    # finder pattern centres are dark, separators light, timing alternates, dark module set
    for cx, cy in ((3, 3), (n - 4, 3), (3, n - 4)):
        assert q.modules[cy][cx] and not q.modules[cy][cx + 2] and q.modules[cy][cx + 3]
    assert [q.modules[6][i] for i in range(8, n - 8)] == [i % 2 == 0 for i in range(8, n - 8)]
    assert q.modules[n - 8][8]


def test_qr_version_selection_and_limits():
    assert QrCode("A" * 14, ec="M").version == 1
    assert QrCode("A" * 15, ec="M").version == 2
    assert QrCode("A" * 150, ec="L").version >= 7      # version information blocks present
    with pytest.raises(ValueError):
        QrCode("A" * 400, ec="H")


def test_qr_png_is_valid():
    png = QrCode("abc").to_png(scale=2, border=4)
    assert png[:8] == b"\x89PNG\r\n\x1a\n"
    ln, typ = struct.unpack("!I4s", png[8:16])
    assert typ == b"IHDR"
    w, h = struct.unpack("!II", png[16:24])
    assert w == h == (21 + 8) * 2
    idat_len = struct.unpack("!I", png[33:37])[0]
    raw = zlib.decompress(png[41:41 + idat_len])
    assert len(raw) == h * (w + 1)


def test_cron_expression():
    c = CronExpression("*/15 9-17 * * 1-5")
    t0 = dt.datetime(2024, 1, 5, 16, 50)        # Friday
    n = dt.datetime.fromtimestamp(c.next_after(int(t0.timestamp() * 1000)) / 1000)
    assert (n.hour, n.minute) == (17, 0)
    n2 = dt.datetime.fromtimestamp(c.next_after(int(dt.datetime(2024, 1, 5, 17, 50).timestamp() * 1000)) / 1000)
    assert n2.weekday() == 0 and (n2.hour, n2.minute) == (9, 0)    # next Monday
    assert CronExpression("0 0 12 * * ?").sets[1] == {12}          # Quartz 6-field form


def test_simple_trigger_repeat_count():
    s = Schedule(token="s", name="s", trigger_type=TriggerType.SimpleTrigger, start_date=1000,
                 trigger_configuration={"repeatInterval": 500, "repeatCount": 2})
    assert next_fire(s, 0, 0) == 1000
    assert next_fire(s, 1000, 1) == 1500
    assert next_fire(s, 1500, 2) == 2000
    assert next_fire(s, 2000, 3) is None
