"""Pure-Python restatement of sha1.go / sha1_efes.go / crc32_efes.go for SMALL cases.

TEST INFRASTRUCTURE ONLY (used by tests/golden/make_golden.py to produce mid-stream
state vectors, and by tests as a third, independent restatement).  Pure-Python loops:
keep inputs to a few KiB.  Citations are /root/reference/<file>:<line>.
"""
from __future__ import annotations

import struct

MASK = 0xFFFFFFFF
IV = (0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476, 0xC3D2E1F0)  # sha1.go:21-25
K = (0x5A827999, 0x6ED9EBA1, 0x8F1BBCDC, 0xCA62C1D6)               # sha1.go:122-127


def _rotl(x: int, n: int) -> int:
    return ((x << n) | (x >> (32 - n))) & MASK


def block(h: list[int], p: bytes) -> None:
    """sha1.go:129-203, in place on h, for every whole 64-byte chunk of p."""
    for off in range(0, len(p) - len(p) % 64, 64):
        w = list(struct.unpack(">16I", p[off:off + 64]))
        a, b, c, d, e = h
        for i in range(80):
            if i >= 16:
                t = w[(i - 3) & 15] ^ w[(i - 8) & 15] ^ w[(i - 14) & 15] ^ w[i & 15]
                w[i & 15] = _rotl(t, 1)
            if i < 20:
                f, k = (b & c) | (~b & d), K[0]
            elif i < 40:
                f, k = b ^ c ^ d, K[1]
            elif i < 60:
                f, k = ((b | c) & d) | (b & c), K[2]
            else:
                f, k = b ^ c ^ d, K[3]
            t = (_rotl(a, 5) + (f & MASK) + e + w[i & 15] + k) & MASK
            a, b, c, d, e = t, a, _rotl(b, 30), c, d
        for i, v in enumerate((a, b, c, d, e)):
            h[i] = (h[i] + v) & MASK


class Sha1Digest:
    """sha1.go:29-34 sha1digest; zero value == Go's `var d sha1digest` (zero IV)."""

    def __init__(self, reset: bool = True):
        self.h = [0] * 5
        self.x = bytearray(64)
        self.nx = 0
        self.len = 0
        if reset:
            self.reset()

    def reset(self) -> None:  # sha1.go:36-44
        self.h = list(IV)
        self.nx = 0
        self.len = 0

    def copy(self) -> "Sha1Digest":
        d = Sha1Digest(reset=False)
        d.h, d.x, d.nx, d.len = list(self.h), bytearray(self.x), self.nx, self.len
        return d

    def write(self, p: bytes) -> int:  # sha1.go:58-79
        n = len(p)
        self.len = (self.len + n) & 0xFFFFFFFFFFFFFFFF
        if self.nx > 0:
            if self.nx > 64:
                raise IndexError("slice bounds out of range")  # Go panic in copy(d.x[d.nx:], p)
            c = min(64 - self.nx, len(p))
            self.x[self.nx:self.nx + c] = p[:c]
            self.nx += c
            if self.nx == 64:
                block(self.h, bytes(self.x))
                self.nx = 0
            p = p[c:]
        if len(p) >= 64:
            m = len(p) & ~63
            block(self.h, p[:m])
            p = p[m:]
        if len(p) > 0:
            self.x[:len(p)] = p
            self.nx = len(p)
        return n

    def sum(self) -> bytes:  # sha1.go:82-120
        d = self.copy()
        ln = d.len
        tmp = bytearray(64)
        tmp[0] = 0x80
        if ln % 64 < 56:
            d.write(bytes(tmp[:56 - ln % 64]))
        else:
            d.write(bytes(tmp[:64 + 56 - ln % 64]))
        d.write(struct.pack(">Q", (ln << 3) & 0xFFFFFFFFFFFFFFFF))
        if d.nx != 0:
            raise RuntimeError("d.nx != 0")  # sha1.go:107-109 panic
        return struct.pack(">5I", *d.h)

    def marshal_text(self) -> str:  # sha1_efes.go:25-38
        b = struct.pack(">5I", *self.h) + bytes(self.x) + struct.pack(">qQ", self.nx, self.len)
        return b.hex()

    def unmarshal_text(self, text: str) -> None:  # sha1_efes.go:40-64
        if len(text) != 200:
            raise ValueError("invalid digest")
        b = bytes.fromhex(text)
        self.h = list(struct.unpack(">5I", b[:20]))
        self.x = bytearray(b[20:84])
        self.nx, self.len = struct.unpack(">qQ", b[84:100])


def crc32_marshal_text(crc: int) -> str:  # crc32_efes.go:18-24
    return struct.pack(">I", crc).hex()
