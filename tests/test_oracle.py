"""The CPU oracle (oracle/efes_oracle.c) pinned against the golden fixtures.

Fixtures come from hashlib/zlib and the reference's own KAT (sha1file_test.go:11-12),
see tests/golden/make_golden.py.  These run without a GPU.
"""
import hashlib
import random
import zlib

import numpy as np
import pytest

from oracle import sha1_ref
from tests.golden.make_golden import synthetic


def test_reference_kat_fox(oracle):
    # sha1file_test.go:10-41 / client_test.go:158-171
    s = oracle.Sha1()
    s.write(b"the quick brown fox jumps over the lazy dog\n")
    assert s.hexdigest() == "5d2781d78fa5a97b7bafa849fe933dfc9dc93eba"


def test_kat_strings(oracle, golden):
    for v in golden["kat"]:
        b = v["text"].encode()
        s = oracle.Sha1()
        s.write(b)
        assert s.hexdigest() == v["sha1"], v["text"]
        c = oracle.Crc32()
        c.write(b)
        assert "%08x" % c.sum32() == v["crc32"], v["text"]


def test_synthetic_generator_matches_numpy(oracle):
    for n, seed in [(0, 1), (1, 2), (7, 3), (8, 4), (1001, 0xEFE5), (65536 + 5, 99)]:
        assert oracle.fill_synthetic(n, seed).tobytes() == synthetic(n, seed)


def test_synthetic_vectors(oracle, golden):
    for v in golden["synthetic"]:
        data = oracle.fill_synthetic(v["length"], v["seed"])
        sha, crc = oracle.hash_message(data)
        assert sha == v["sha1"], v["length"]
        assert "%08x" % crc == v["crc32"], v["length"]


def test_sha1_state_vectors(oracle, golden):
    """MarshalText after every Write (sha1_efes.go:25-38), stale x bytes included."""
    for case in golden["sha1_states"]:
        s = oracle.Sha1(reset=case["reset"])
        for w, text in zip(case["writes"], case["texts"]):
            assert s.write(bytes.fromhex(w)) == 0
            assert s.marshal_text() == text, case["name"]
        assert s.hexdigest() == case["sum"], case["name"]


def test_sha1_partial_digest_roundtrip(oracle):
    """sha1_efes_test.go:8-29: zero-valued digest, Write, Marshal, Unmarshal, same Sum."""
    d = oracle.Sha1(reset=False)
    d.write(b"hello world")
    hex1 = d.hexdigest()
    d2 = oracle.Sha1(reset=False)
    assert d2.unmarshal_text(d.marshal_text()) == 0
    assert d2.hexdigest() == hex1 == "73e8730e5086d8ced928b654beeb0e5383f9be01"


def test_crc32_partial_digest_roundtrip(oracle, golden):
    """crc32_efes_test.go:8-29 + fixture texts."""
    for case in golden["crc32_states"]:
        c = oracle.Crc32()
        for w, text in zip(case["writes"], case["texts"]):
            c.write(bytes.fromhex(w))
            assert c.marshal_text() == text
        assert c.sum32() == case["sum32"]
        c2 = oracle.Crc32()
        assert c2.unmarshal_text(c.marshal_text()) == 0
        assert c2.sum32() == c.sum32()


def test_unmarshal_errors(oracle):
    s = oracle.Sha1()
    assert s.unmarshal_text("00" * 99) == oracle.ERR_INVALID_DIGEST
    assert s.unmarshal_text("zz" + "00" * 99) == oracle.ERR_INVALID_DIGEST
    assert s.unmarshal_text("AB" * 100) == 0  # Go's hex.Decode accepts upper case
    c = oracle.Crc32()
    assert c.unmarshal_text("1234567") == oracle.ERR_INVALID_DIGEST
    assert c.unmarshal_text("1234567g") == oracle.ERR_INVALID_DIGEST


def test_panics_become_errors(oracle):
    s = oracle.Sha1()
    s.unmarshal_text(s.marshal_text()[:168] + "%016x" % 65 + "%016x" % 0)
    assert s.write(b"x") == oracle.ERR_PANIC          # copy(d.x[65:]) panics
    s = oracle.Sha1()
    s.unmarshal_text(s.marshal_text()[:168] + "%016x" % 3 + "%016x" % 0)  # nx=3 but len=0
    assert s.sum()[0] == oracle.ERR_PANIC             # checkSum: d.nx != 0


def test_nx64_and_negative_nx_follow_go(oracle):
    # nx == 64 is a full pending block: the next Write compresses it (sha1.go:62-67)
    a = oracle.Sha1()
    a.write(b"A" * 64)
    ref = a.hexdigest()
    b = oracle.Sha1()
    t = b.marshal_text()
    b.unmarshal_text(t[:40] + (b"A" * 64).hex() + "%016x" % 64 + "%016x" % 64)
    assert b.write(b"") == 0 and b.nx == 0
    assert b.hexdigest() == ref
    # pure-Python restatement agrees on these quirks
    p = sha1_ref.Sha1Digest()
    p.unmarshal_text(t[:40] + (b"A" * 64).hex() + "%016x" % 64 + "%016x" % 64)
    p.write(b"")
    assert p.sum().hex() == ref


def test_random_splits_agree_with_restatement(oracle):
    rng = random.Random(5)
    for k in range(40):
        n = rng.randint(0, 700)
        data = synthetic(n, 1000 + k)
        cuts = sorted(rng.sample(range(n + 1), min(3, n + 1)))
        o, p = oracle.Sha1(), sha1_ref.Sha1Digest()
        prev = 0
        for c in cuts + [n]:
            o.write(data[prev:c])
            p.write(data[prev:c])
            prev = c
            assert o.marshal_text() == p.marshal_text()
        assert o.hexdigest() == p.sum().hex() == hashlib.sha1(data).hexdigest()


def test_crc_slicing_equals_simple(oracle):
    rng = np.random.default_rng(3)
    for n in [0, 1, 8, 15, 16, 17, 100, 4097]:
        a = rng.integers(0, 256, n, dtype=np.uint8)
        L = oracle.lib()
        s = L.oracle_crc32_slicing_update(0x12345678, a.ctypes.data, n)
        t = L.oracle_crc32_simple_update(0x12345678, a.ctypes.data, n)
        assert s == t == zlib.crc32(a.tobytes(), 0x12345678)


def test_sha1file_script(oracle, golden):
    """sha1file_test.go:31-39 seek/read script."""
    f = golden["sha1file"]
    sf = oracle.Sha1File(f["content"].encode())
    for (seek, n), want in zip(f["script"], f["reads"]):
        assert sf.seek(seek, 0) == seek
        assert sf.read(n).decode() == want
    assert sf.sum().hex() == f["sha1"]


def test_sha1file_errors(oracle):
    sf = oracle.Sha1File(b"0123456789")
    assert sf.read(4) == b"0123"
    with pytest.raises(IOError, match="seeking forward"):
        sf.seek(6, 0)
    # Go moved the underlying reader but not f.position: next Read hashes bytes 6.. as 4..
    assert sf.read(2) == b"67"
    sf2 = oracle.Sha1File(b"0123456789")
    sf2.read(3)
    sf2.seek(0, 0)
    sf2.read(1)
    sf2.st.position = 5  # positioned past the hashed prefix
    with pytest.raises(IOError, match="missing data"):
        sf2.read(1)


def test_hash_many_threads(oracle):
    n, size = 6, 10000
    buf = oracle.fill_synthetic(n * size, 77)
    secs, sha, crc = oracle.hash_many(buf, size, np.full(n, size - 3), 3)
    for i in range(n):
        m = buf[i * size:i * size + size - 3].tobytes()
        assert bytes(sha[i]).hex() == hashlib.sha1(m).hexdigest()
        assert crc[i] == zlib.crc32(m)
    assert secs >= 0


def test_chunksize_mirrors_go():
    """chunksize.go Set/String semantics (benchmark size classes come from these)."""
    from efes_amd import chunksize as c
    assert c.parse("1M") == 1 << 20 and c.parse("50M") == 50 << 20 and c.parse("64K") == 65536
    assert c.parse("0") == 0 and c.parse("123") == 123 and c.parse("2G") == 2 << 30 and c.parse("-1K") == -1024
    assert c.parse("9223372036854775807K") == -1024  # int64 wrap-around of i *= K
    for bad in ("1.5M", "M", "1 M", "x", "1KB", "99999999999999999999"):
        with pytest.raises(ValueError):
            c.parse(bad)
    with pytest.raises(IndexError):
        c.parse("")
    assert [c.format(v) for v in (0, 1536, 2048, 1 << 20, 3 << 30, -2048, 1)] == \
        ["0", "1536", "2K", "1M", "3G", "-2K", "1"]
    assert [c.format(v) for v in c.MIXED_CLASSES] == ["64K", "128K", "256K", "512K", "1M", "2M", "4M", "8M",
                                                       "16M", "32M", "64M"]
