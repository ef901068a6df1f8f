"""The span CRC's decomposition (efes_crc_span.hip), restated in Python and checked against zlib on
the CPU: rows of L lines dealt round-robin over G workgroups, each lane folding its lines with
Horner's rule under the stride operator x^(8*64*L*G), then advanced over what follows its last
line -- the rest of that row (lane_op), the rows, extra lines and rest bytes after it (op[w], as the
launcher computes it), or for the partial last row lane_op[extra-1-j] and the rest bytes.  Small L
and G so every case runs in milliseconds; the GPU tests (tests/test_gpu_span.py) check the kernel."""
import random
import zlib

POLY = 0xEDB88320  # crc32.go:30, reflected


def mulmod(a: int, b: int) -> int:
    """a * b mod P in the reflected representation (bit 31 = x^0), as gf2_mulmod."""
    p = 0
    for i in range(32):
        if (a >> (31 - i)) & 1:
            p ^= b
        b = (b >> 1) ^ (POLY if b & 1 else 0)
    return p


def xpow8n(n: int) -> int:
    """x^(8n) mod P (xpow8n in efes_crc_span.hip)."""
    x2n = [1 << 30]
    for _ in range(31):
        x2n.append(mulmod(x2n[-1], x2n[-1]))
    p, k = 1 << 31, 3
    while n:
        if n & 1:
            p = mulmod(x2n[k & 31], p)
        n >>= 1
        k += 1
    return p


def raw(data: bytes) -> int:
    """The raw register after `data` from zero (no pre/post inversion)."""
    crc = 0
    for b in data:
        crc ^= b
        for _ in range(8):
            crc = (crc >> 1) ^ (POLY if crc & 1 else 0)
    return crc


def span_round_robin(buf: bytes, crc_in: int, L: int, G: int, line: int = 64) -> int:
    """crc32digest.Write of buf from state crc_in (head = 0: buf starts 16-byte aligned)."""
    n = len(buf)
    nline, rest = n // line, n % line
    # span_prep_kernel: ~(Z^n(~crc) ^ raw(rest)); every bulk contribution is XORed into it
    state = (~mulmod(xpow8n(n), ~crc_in & 0xFFFFFFFF)) & 0xFFFFFFFF ^ raw(buf[nline * line:])
    rtot, extra = nline // L, nline % L
    stride = xpow8n(line * L * G)
    zrow, base = xpow8n(line * L), xpow8n(line * extra + rest)
    lane_op = [xpow8n(line * k) for k in range(L)]
    op = []
    for w in range(G):  # the launcher's op[w]
        d = (rtot - 1 - w) % G
        p = 1 << 31
        for _ in range(d):
            p = mulmod(zrow, p)
        op.append(mulmod(base, p) if w < rtot else 0)
    for w in range(G):
        rows = (rtot - 1 - w) // G + 1 if rtot > w else 0
        for j in range(L):
            acc = 0
            for k in range(rows):
                li = (w + k * G) * L + j
                acc = mulmod(stride, acc) ^ raw(buf[li * line:(li + 1) * line])
            if rtot % G == w and j < extra:
                li = rtot * L + j
                acc = mulmod(stride, acc) ^ raw(buf[li * line:(li + 1) * line])
                c = mulmod(xpow8n(rest), mulmod(lane_op[extra - 1 - j], acc))
            elif rows:
                c = mulmod(op[w], mulmod(lane_op[L - 1 - j], acc))
            else:
                c = 0
            state ^= c
    return state


def test_round_robin_decomposition_matches_zlib():
    rng = random.Random(5)
    for L, G in [(1, 1), (2, 1), (4, 3), (3, 5), (8, 4), (5, 7)]:
        for _ in range(4):
            n = rng.randrange(0, 64 * L * (3 * G + 2) + 200)
            buf = bytes(rng.getrandbits(8) for _ in range(n))
            crc_in = rng.getrandbits(32)
            assert span_round_robin(buf, crc_in, L, G) == zlib.crc32(buf, crc_in), (L, G, n)
