"""GPU parity of the span CRC (efes_crc32_span): CRC-32 of one long device
buffer computed segment-parallel over the whole GPU must equal crc32.go's serial Write
(crc32.go:76-86) of the same bytes -- the oracle's C restatement for small cases, zlib.crc32 (the
same IEEE algorithm, pinned against the oracle in test_oracle.py) at sizes the oracle would take
long on, and size-independent properties (chained calls = one call, pieces merged by
efes_crc32_combine = one call) at full size.  Bit-exact."""
import random
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from efes_amd import hashing
    from oracle import oracle
    return dict(torch=torch, hashing=hashing, ctx=hashing.default_context(0), oracle=oracle)


def _span(env, buf, off: int, n: int, crc_in: int = 0) -> int:
    """efes_crc32_span of buf[off:off+n] into a device state holding crc_in."""
    torch = env["torch"]
    st = torch.tensor([crc_in], dtype=torch.int64, device="cuda:0")  # the state is its low 4 bytes
    env["ctx"].crc32_span(buf.data_ptr() + off, n, st.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return int(st.item()) & 0xFFFFFFFF


def _device_bytes(env, nbytes: int, seed: int):
    torch = env["torch"]
    buf = torch.empty(nbytes, dtype=torch.uint8, device="cuda:0")
    env["ctx"].fill_synthetic(buf.data_ptr(), nbytes - nbytes % 8, seed, torch.cuda.current_stream().cuda_stream)
    if nbytes % 8:
        buf[nbytes - nbytes % 8:] = 0x5A
    torch.cuda.synchronize()
    return buf


# lengths around every boundary of the decomposition: the 16-byte head, the < 64-byte rest,
# 64-byte lines, one workgroup row (1024 lines = 64 KiB), partial and whole rows, several rows
# per lane, ragged workgroup ranges (and the 128-byte / 128 KiB edges of other line sizes)
LENGTHS = [0, 1, 15, 16, 17, 63, 64, 65, 79, 80, 81, 127, 128, 129, 143, 144, 1000, 4095, 4096, 4097,
           32768 + 5, 65535, 65536, 65537, 65536 + 64 * 7 + 5, 131071, 131072, 131073, 131072 + 128 * 7 + 5,
           262144 + 3, 524288 + 127, (1 << 20) + 13, 3 * (1 << 20) - 1]


def test_span_matches_oracle_small(env):
    """Every length and misalignment 0..15 against the oracle's crc32digest, from fresh and mid-stream states."""
    oracle = env["oracle"]
    total = max(LENGTHS) + 64
    buf = _device_bytes(env, total, 0x5BA7)
    host = buf.cpu().numpy()
    rng = random.Random(11)
    for n in LENGTHS:
        for off in (0, 1, 7, 15) if n > 4096 else range(16):
            o = oracle.Crc32()
            crc_in = rng.choice([0, 0xFFFFFFFF, rng.getrandbits(32)])
            o.st.crc = crc_in
            o.write(host[off:off + n].tobytes())
            got = _span(env, buf, off, n, crc_in)
            assert got == o.sum32(), (n, off, hex(crc_in), hex(got), hex(o.sum32()))


def test_span_matches_zlib_many_workgroups(env):
    """Sizes that spread over hundreds of workgroups with ragged ranges (nblk not a multiple of the
    workgroup count), misaligned, against zlib."""
    buf = _device_bytes(env, (300 << 20) + 4096, 0xC0FFEE)
    host = buf.cpu().numpy()
    for off, n in [(0, 300 << 20), (3, (300 << 20) - 7), (9, (137 << 20) + 12345), (0, (64 << 20) + 64 * 513 + 1)]:
        exp = zlib.crc32(host[off:off + n])
        assert _span(env, buf, off, n) == exp, (off, n)


def test_span_chained_and_combined_full_size(env):
    """4 GiB + 5 bytes: one call == random pieces chained through one state == pieces on separate
    states merged with efes_crc32_combine (the multi-GPU gather); zlib at the end."""
    n = (4 << 30) + 5
    buf = _device_bytes(env, n, 0x10B)
    whole = _span(env, buf, 0, n)
    rng = random.Random(5)
    cuts = sorted(rng.sample(range(1, n), 6))
    bounds = [0] + cuts + [n]
    chained = 0
    merged = None
    for a, b in zip(bounds, bounds[1:]):
        chained = _span(env, buf, a, b - a, chained)
        part = _span(env, buf, a, b - a)
        merged = part if merged is None else env["hashing"].crc32_combine(merged, part, b - a)
    assert chained == whole and merged == whole
    # zlib over the host copy, in 1 GiB pieces
    crc = 0
    for a in range(0, n, 1 << 30):
        crc = zlib.crc32(buf[a:min(n, a + (1 << 30))].cpu().numpy(), crc)
    assert whole == crc


def test_span_zero_bytes_and_constant_data(env):
    """All-zero and all-0xFF buffers (the CRC's fixed-pattern cases), 16 MiB + 3, against zlib."""
    torch = env["torch"]
    n = (16 << 20) + 3
    for v in (0, 0xFF):
        buf = torch.full((n,), v, dtype=torch.uint8, device="cuda:0")
        assert _span(env, buf, 0, n) == zlib.crc32(bytes([v]) * n)
        assert _span(env, buf, 1, n - 1, 0x12345678) == zlib.crc32(bytes([v]) * (n - 1), 0x12345678)


def test_span_concurrent_streams_and_null(env):
    """Calls on different streams at once keep their states apart (no shared scratch: every
    workgroup XORs into its own call's state); length 0 with a NULL pointer leaves the state."""
    torch = env["torch"]
    n = (64 << 20) + 77
    bufs = [_device_bytes(env, n, 100 + i) for i in range(4)]
    expect = [zlib.crc32(b.cpu().numpy(), 7 * i) for i, b in enumerate(bufs)]
    streams = [torch.cuda.Stream(device="cuda:0") for _ in bufs]
    states = [torch.tensor([7 * i], dtype=torch.int64, device="cuda:0") for i in range(len(bufs))]
    torch.cuda.synchronize()
    for rep in range(3):
        for i, (b, s, st) in enumerate(zip(bufs, streams, states)):
            with torch.cuda.stream(s):
                st.fill_(7 * i)
                env["ctx"].crc32_span(b.data_ptr(), n, st.data_ptr(), s.cuda_stream)
        torch.cuda.synchronize()
        assert [int(st.item()) & 0xFFFFFFFF for st in states] == expect, rep
    st = torch.tensor([0xCAFEF00D], dtype=torch.int64, device="cuda:0")
    torch.cuda.synchronize()  # the call below runs on the context's own (non-blocking) stream
    env["ctx"].crc32_span(0, 0, st.data_ptr(), None)
    env["ctx"].sync()
    assert int(st.item()) == 0xCAFEF00D


def test_span_pieces_on_two_contexts_combine(env):
    """One object over two contexts (standing in for two GPUs, efes_amd/shard.py): each spans its
    piece from a zero state, the 4-byte results fold in piece order == one call == zlib."""
    from efes_amd.hashing import Context
    from efes_amd.shard import combine_piece_crcs, piece_bounds
    torch = env["torch"]
    n = (96 << 20) + 4097
    buf = _device_bytes(env, n, 0xAB)
    ctxs = [env["ctx"], Context(0)]
    try:
        pieces = []
        for ctx, (a, m) in zip(ctxs, piece_bounds(n, 2)):
            st = torch.zeros(1, dtype=torch.int64, device="cuda:0")
            torch.cuda.synchronize()
            ctx.crc32_span(buf.data_ptr() + a, m, st.data_ptr(), None)
            ctx.sync()
            pieces.append((int(st.item()) & 0xFFFFFFFF, m))
        whole = _span(env, buf, 0, n)
        assert combine_piece_crcs(pieces) == whole == zlib.crc32(buf.cpu().numpy())
    finally:
        ctxs[1].close()


def test_span_random_lengths_against_zlib(env):
    """Seeded random lengths from 1 byte to 320 MiB (every workgroup count from 1 to the CU count,
    partial last rows owned by any workgroup of the round-robin), random starts and states."""
    n_max = 320 << 20
    buf = _device_bytes(env, n_max + 64, 0x5EED)
    host = buf.cpu().numpy()
    rng = random.Random(2026)
    for _ in range(48):
        n = int(rng.choice([rng.randrange(1, 1 << 20), rng.randrange(1 << 20, 64 << 20), rng.randrange(64 << 20, n_max)]))
        off = rng.randrange(0, 16)
        crc_in = rng.getrandbits(32)
        assert _span(env, buf, off, n, crc_in) == zlib.crc32(host[off:off + n], crc_in), (n, off, hex(crc_in))
