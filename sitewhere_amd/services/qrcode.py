"""QR Code (ISO/IEC 18004) encoder -- byte mode, versions 1-10, EC levels L/M/Q/H -- and a PNG writer.

Reference: ``service-label-generation/.../labels/symbology/QrCodeGenerator.java:37-70`` (ZXing).
ZXing is not available, so the symbology is implemented here: Reed-Solomon over GF(256)/0x11D,
block interleaving, function patterns, zig-zag placement, the 8 masks with penalty scoring, BCH
format/version information.
"""
from __future__ import annotations

import struct
import zlib

# (ec codewords per block, blocks in group 1, data cw per g1 block, blocks in group 2, data cw per g2 block)
EC_TABLE = {
    "L": [(7, 1, 19, 0, 0), (10, 1, 34, 0, 0), (15, 1, 55, 0, 0), (20, 1, 80, 0, 0), (26, 1, 108, 0, 0),
          (18, 2, 68, 0, 0), (20, 2, 78, 0, 0), (24, 2, 97, 0, 0), (30, 2, 116, 0, 0), (18, 2, 68, 2, 69)],
    "M": [(10, 1, 16, 0, 0), (16, 1, 28, 0, 0), (26, 1, 44, 0, 0), (18, 2, 32, 0, 0), (24, 2, 43, 0, 0),
          (16, 4, 27, 0, 0), (18, 4, 31, 0, 0), (22, 2, 38, 2, 39), (22, 3, 36, 2, 37), (26, 4, 43, 1, 44)],
    "Q": [(13, 1, 13, 0, 0), (22, 1, 22, 0, 0), (18, 2, 17, 0, 0), (26, 2, 24, 0, 0), (18, 2, 15, 2, 16),
          (24, 4, 19, 0, 0), (18, 2, 14, 4, 15), (22, 4, 18, 2, 19), (20, 4, 16, 4, 17), (24, 6, 19, 2, 20)],
    "H": [(17, 1, 9, 0, 0), (28, 1, 16, 0, 0), (22, 2, 13, 0, 0), (16, 4, 9, 0, 0), (22, 2, 11, 2, 12),
          (28, 4, 15, 0, 0), (26, 4, 13, 1, 14), (26, 4, 14, 2, 15), (24, 4, 12, 4, 13), (28, 6, 15, 2, 16)],
}
FORMAT_EC = {"L": 1, "M": 0, "Q": 3, "H": 2}
ALIGN = {1: [], 2: [6, 18], 3: [6, 22], 4: [6, 26], 5: [6, 30], 6: [6, 34], 7: [6, 22, 38], 8: [6, 24, 42],
         9: [6, 26, 46], 10: [6, 28, 50]}


def gf_mul(x: int, y: int) -> int:
    z = 0
    for i in reversed(range(8)):
        z = (z << 1) ^ ((z >> 7) * 0x11D)
        z ^= ((y >> i) & 1) * x
    return z


def rs_divisor(degree: int) -> list[int]:
    result = [0] * (degree - 1) + [1]
    root = 1
    for _ in range(degree):
        for j in range(degree):
            result[j] = gf_mul(result[j], root)
            if j + 1 < degree:
                result[j] ^= result[j + 1]
        root = gf_mul(root, 0x02)
    return result


def rs_remainder(data, divisor) -> list[int]:
    result = [0] * len(divisor)
    for b in data:
        factor = b ^ result.pop(0)
        result.append(0)
        for i, coef in enumerate(divisor):
            result[i] ^= gf_mul(coef, factor)
    return result


def data_capacity(version: int, ec: str) -> int:
    _, b1, d1, b2, d2 = EC_TABLE[ec][version - 1]
    return b1 * d1 + b2 * d2


class QrCode:
    def __init__(self, data: bytes | str, ec: str = "M", min_version: int = 1, mask: int | None = None):
        if isinstance(data, str):
            data = data.encode("utf-8")
        self.ec = ec
        for v in range(min_version, 11):
            cc_bits = 8 if v < 10 else 16
            if 4 + cc_bits + 8 * len(data) <= data_capacity(v, ec) * 8:
                break
        else:
            raise ValueError("data too long for QR versions 1-10")
        self.version = v
        self.size = 17 + 4 * v
        n = self.size
        self.modules = [[False] * n for _ in range(n)]
        self.function = [[False] * n for _ in range(n)]
        self._draw_function_patterns()
        codewords = self._codewords(data, cc_bits)
        self._place(codewords)
        if mask is None:
            best, mask = None, 0
            for m in range(8):
                self._apply_mask(m)
                self._draw_format(m)
                p = self.penalty()
                if best is None or p < best:
                    best, mask = p, m
                self._apply_mask(m)
        self.mask = mask
        self._apply_mask(mask)
        self._draw_format(mask)

    # ---- function patterns --------------------------------------------------------------
    def _set(self, x, y, dark):
        self.modules[y][x] = dark
        self.function[y][x] = True

    def _draw_function_patterns(self):
        n = self.size
        for i in range(n):
            self._set(6, i, i % 2 == 0)
            self._set(i, 6, i % 2 == 0)
        for (cx, cy) in ((3, 3), (n - 4, 3), (3, n - 4)):
            for dy in range(-4, 5):
                for dx in range(-4, 5):
                    x, y = cx + dx, cy + dy
                    if 0 <= x < n and 0 <= y < n:
                        self._set(x, y, max(abs(dx), abs(dy)) not in (2, 4))
        pos = ALIGN[self.version]
        last = len(pos) - 1
        for i, ax in enumerate(pos):
            for j, ay in enumerate(pos):
                if (i == 0 and j == 0) or (i == 0 and j == last) or (i == last and j == 0):
                    continue
                for dy in range(-2, 3):
                    for dx in range(-2, 3):
                        self._set(ax + dx, ay + dy, max(abs(dx), abs(dy)) != 1)
        self._draw_format(0)
        if self.version >= 7:
            rem = self.version
            for _ in range(12):
                rem = (rem << 1) ^ ((rem >> 11) * 0x1F25)
            bits = self.version << 12 | rem
            for i in range(18):
                bit = (bits >> i) & 1 == 1
                a, b = n - 11 + i % 3, i // 3
                self._set(a, b, bit)
                self._set(b, a, bit)

    def _draw_format(self, mask: int):
        data = FORMAT_EC[self.ec] << 3 | mask
        rem = data
        for _ in range(10):
            rem = (rem << 1) ^ ((rem >> 9) * 0x537)
        bits = (data << 10 | rem) ^ 0x5412
        self.format_bits = bits
        n = self.size

        def bit(i):
            return (bits >> i) & 1 == 1
        for i in range(6):
            self._set(8, i, bit(i))
        self._set(8, 7, bit(6))
        self._set(8, 8, bit(7))
        self._set(7, 8, bit(8))
        for i in range(9, 15):
            self._set(14 - i, 8, bit(i))
        for i in range(8):
            self._set(n - 1 - i, 8, bit(i))
        for i in range(8, 15):
            self._set(8, n - 15 + i, bit(i))
        self._set(8, n - 8, True)  # dark module

    # ---- data -------------------------------------------------------------------------------
    def _codewords(self, data: bytes, cc_bits: int) -> list[int]:
        ecw, b1, d1, b2, d2 = EC_TABLE[self.ec][self.version - 1]
        cap = (b1 * d1 + b2 * d2) * 8
        bits = [0, 1, 0, 0]
        bits += [(len(data) >> i) & 1 for i in reversed(range(cc_bits))]
        for byte in data:
            bits += [(byte >> i) & 1 for i in reversed(range(8))]
        bits += [0] * min(4, cap - len(bits))
        bits += [0] * (-len(bits) % 8)
        cw = [int("".join(map(str, bits[i:i + 8])), 2) for i in range(0, len(bits), 8)]
        pad = 0xEC
        while len(cw) * 8 < cap:
            cw.append(pad)
            pad ^= 0xEC ^ 0x11
        blocks, k = [], 0
        for count, size in ((b1, d1), (b2, d2)):
            for _ in range(count):
                blocks.append(cw[k:k + size])
                k += size
        div = rs_divisor(ecw)
        ecs = [rs_remainder(b, div) for b in blocks]
        out = []
        for i in range(max(len(b) for b in blocks)):
            out += [b[i] for b in blocks if i < len(b)]
        for i in range(ecw):
            out += [e[i] for e in ecs]
        self.blocks, self.ec_blocks = blocks, ecs
        return out

    def _place(self, cw: list[int]):
        n = self.size
        i, total = 0, len(cw) * 8
        right = n - 1
        while right >= 1:
            if right == 6:
                right = 5
            for vert in range(n):
                for j in range(2):
                    x = right - j
                    upward = ((right + 1) & 2) == 0
                    y = n - 1 - vert if upward else vert
                    if not self.function[y][x] and i < total:
                        self.modules[y][x] = (cw[i >> 3] >> (7 - (i & 7))) & 1 == 1
                        i += 1
            right -= 2

    @staticmethod
    def _mask_fn(m):
        return [lambda x, y: (x + y) % 2 == 0, lambda x, y: y % 2 == 0, lambda x, y: x % 3 == 0,
                lambda x, y: (x + y) % 3 == 0, lambda x, y: (x // 3 + y // 2) % 2 == 0,
                lambda x, y: x * y % 2 + x * y % 3 == 0, lambda x, y: (x * y % 2 + x * y % 3) % 2 == 0,
                lambda x, y: ((x + y) % 2 + x * y % 3) % 2 == 0][m]

    def _apply_mask(self, m: int):
        f = self._mask_fn(m)
        for y in range(self.size):
            for x in range(self.size):
                if not self.function[y][x] and f(x, y):
                    self.modules[y][x] = not self.modules[y][x]

    def penalty(self) -> int:
        n, M = self.size, self.modules
        score = 0
        lines = [M[y] for y in range(n)] + [[M[y][x] for y in range(n)] for x in range(n)]
        finder = [True, False, True, True, True, False, True]
        for line in lines:
            run, prev = 0, None
            for c in line:
                if c == prev:
                    run += 1
                else:
                    if run >= 5:
                        score += 3 + (run - 5)
                    run, prev = 1, c
            if run >= 5:
                score += 3 + (run - 5)
            for i in range(n - 6):
                if line[i:i + 7] == finder:
                    before = line[max(0, i - 4):i]
                    after = line[i + 7:i + 11]
                    if (len(before) == 4 and not any(before)) or (len(after) == 4 and not any(after)):
                        score += 40
        for y in range(n - 1):
            for x in range(n - 1):
                c = M[y][x]
                if c == M[y][x + 1] == M[y + 1][x] == M[y + 1][x + 1]:
                    score += 3
        dark = sum(map(sum, M))
        k = abs(dark * 20 - n * n * 10) // (n * n)
        return score + k * 10

    # ---- output -------------------------------------------------------------------------------
    def to_text(self) -> str:
        return "\n".join("".join("##" if c else "  " for c in row) for row in self.modules)

    def to_png(self, scale: int = 8, border: int = 4) -> bytes:
        n = self.size
        w = (n + 2 * border) * scale
        rows = []
        white = b"\xff"
        for y in range(-border, n + border):
            row = bytearray()
            for x in range(-border, n + border):
                dark = 0 <= x < n and 0 <= y < n and self.modules[y][x]
                row += (b"\x00" if dark else white) * scale
            for _ in range(scale):
                rows.append(b"\x00" + bytes(row))
        raw = zlib.compress(b"".join(rows), 9)

        def chunk(t, d):
            return struct.pack("!I", len(d)) + t + d + struct.pack("!I", zlib.crc32(t + d) & 0xFFFFFFFF)
        return (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack("!IIBBBBB", w, w, 8, 0, 0, 0, 0)) +
                chunk(b"IDAT", raw) + chunk(b"IEND", b""))


def decode_format_bits(bits: int) -> tuple[str, int] | None:
    """Inverse of the format BCH code (used by the tests to read a symbol back)."""
    for ec, e in FORMAT_EC.items():
        for m in range(8):
            data = e << 3 | m
            rem = data
            for _ in range(10):
                rem = (rem << 1) ^ ((rem >> 9) * 0x537)
            if ((data << 10 | rem) ^ 0x5412) == bits:
                return ec, m
    return None
