"""Fused CRC + SHA-1 digest pairs (efes_stream.cpp, efes_hash.h ABI 6) against the CPU oracle.

io.MultiWriter(f, CRC32, Sha1) (filereceiver.go:208-209) hands every body buffer to the CRC digest
and then, unchanged, to the SHA-1 digest (fileinfo.go:20-27 makes the two).  The library binds such
a pair to ONE upload keeping both hashes: the CRC Write is staged and held, the SHA-1 Write of the
same (p, n) is checked against the staged bytes (memcmp) and confirms it.  Everything else must
split the pair without changing a single result, so these tests drive pairs that DIVERGE in every
way the Go surface allows -- a Write to one digest only, the SHA-1 digest written first, the same
pointer with other bytes (the buffer changed between the two Writes) or another length, empty
Writes, Writes larger than a staging chunk, Reset / UnmarshalText / MarshalText / Sum of either
member first, a member freed mid-stream, evictions of pairs on a 15-slot queue -- from 16 threads,
and compare every text and digest with the oracle doing the same Writes.  The pure MultiWriter
pattern must fuse completely: every byte hashed once (queue byte counter = body bytes).
"""
import ctypes
import hashlib
import os
import random
import subprocess
import sys
import threading
import zlib

import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import efes_amd
    from efes_amd import _lib, hashing
    return dict(efes=efes_amd, hashing=hashing, lib=_lib.lib(), check=_lib.check)


def _stats(gpu):
    return gpu["hashing"].pair_stats()


def _delta(a, b):
    return {k: b[k] - a[k] for k in a}


class Obj:
    """One object's two digests (a FileInfo's Digest) and the oracle's, written through raw
    pointers so a test controls which address each Write passes."""

    def __init__(self, gpu, oracle, ctx=None, pool=None):
        self.g = gpu
        h = gpu["hashing"]
        self.sha = h.Sha1Digest(ctx, pool=pool)
        self.crc = h.CRC32Digest(ctx, pool=pool)
        self.osha = oracle.Sha1()
        self.ocrc = oracle.Crc32()
        self.oracle = oracle

    def crc_write(self, buf, off, n):
        assert off + n <= len(buf)
        self.g["check"](self.g["lib"].efes_crc32_write(self.crc._h, ctypes.addressof(buf) + off, n), "crc write")
        self.ocrc.write(bytes(buf[off:off + n]))

    def sha_write(self, buf, off, n):
        assert off + n <= len(buf)
        self.g["check"](self.g["lib"].efes_sha1_write(self.sha._h, ctypes.addressof(buf) + off, n), "sha write")
        assert self.osha.write(bytes(buf[off:off + n])) == 0

    def check_texts(self, sha_first=True, tag=""):
        if sha_first:
            st, ct = self.sha.marshal_text().decode(), self.crc.marshal_text().decode()
        else:
            ct, st = self.crc.marshal_text().decode(), self.sha.marshal_text().decode()
        assert st == self.osha.marshal_text(), ("sha1 text", tag)
        assert ct == self.ocrc.marshal_text(), ("crc32 text", tag)

    def check_sums(self, sha_first=True, tag=""):
        if sha_first:
            s, c = self.sha.sum(), self.crc.sum32()
        else:
            c, s = self.crc.sum32(), self.sha.sum()
        rc, want = self.osha.sum()
        assert rc == 0 and s == want, ("sha1 sum", tag)
        assert c == self.ocrc.sum32(), ("crc32 sum", tag)


def _buf(n: int, seed: int):
    b = (ctypes.c_uint8 * max(n, 1))()
    ctypes.memmove(b, random.Random(seed).randbytes(n), n)
    return b


OPS = ["mw", "mw", "mw", "mw", "crc_only", "sha_only", "mutated", "other_len", "sha_first", "empty_sha",
       "reset_sha", "reset_crc", "unmarshal_sha", "unmarshal_crc", "texts_sha_first", "texts_crc_first",
       "sum_sha_first", "sum_crc_first", "big", "mw_two_buffers"]


def _script(gpu, oracle, rng: random.Random, steps: int, ctx=None, pool=None, tag=""):
    """A random sequence of Go-surface calls on one object; every sync point compared with the oracle."""
    o = Obj(gpu, oracle, ctx, pool)
    size = 800_000  # every Write stays inside: off < 430 000, n <= 365 536
    buf = _buf(size, rng.randrange(1 << 30))
    for k in range(steps):
        op = rng.choice(OPS)
        n = rng.choice([1, 55, 64, 4096, 32768, 32768, 40000, 65536])
        off = rng.randrange(0, size - 370_000)
        t = f"{tag} step {k} {op} n={n}"
        if op == "mw":  # the MultiWriter pattern: CRC then SHA-1, same (p, n)
            o.crc_write(buf, off, n)
            o.sha_write(buf, off, n)
        elif op == "crc_only":
            o.crc_write(buf, off, n)
        elif op == "sha_only":
            o.sha_write(buf, off, n)
        elif op == "mutated":  # same pointer, the buffer changed between the two Writes
            o.crc_write(buf, off, n)
            # the first / last 64 bytes or anywhere: the fused compare-and-stage has a head, a
            # 64-byte body loop and a tail
            at = rng.choice([rng.randrange(min(n, 64)), n - 1 - rng.randrange(min(n, 64)), rng.randrange(n)])
            buf[off + at] ^= 1 + rng.randrange(255)
            o.sha_write(buf, off, n)
        elif op == "other_len":
            o.crc_write(buf, off, n)
            o.sha_write(buf, off, max(0, n - 1 - rng.randrange(3)))
        elif op == "sha_first":
            o.sha_write(buf, off, n)
            o.crc_write(buf, off, n)
        elif op == "empty_sha":
            o.crc_write(buf, off, n)
            o.sha_write(buf, off, 0)
            o.sha_write(buf, off, n)
        elif op == "reset_sha":
            o.crc_write(buf, off, n)
            o.sha.reset()
            gpu["oracle_lib"].oracle_sha1_reset(ctypes.byref(o.osha.st))
            o.sha_write(buf, off, n)
        elif op == "reset_crc":
            o.crc_write(buf, off, n)
            o.crc.reset()
            o.ocrc = oracle.Crc32()
            o.sha_write(buf, off, n)
        elif op == "unmarshal_sha":  # a resumed PATCH: the .info state of another object
            other = oracle.Sha1()
            other.write(bytes(buf[off:off + rng.randrange(1, 200)]))
            txt = other.marshal_text()
            o.sha.unmarshal_text(txt)
            o.osha.unmarshal_text(txt)
        elif op == "unmarshal_crc":
            other = oracle.Crc32()
            other.write(bytes(buf[off:off + 77]))
            txt = other.marshal_text()
            o.crc.unmarshal_text(txt)
            o.ocrc.unmarshal_text(txt)
        elif op == "texts_sha_first":
            o.check_texts(True, t)
        elif op == "texts_crc_first":
            o.check_texts(False, t)
        elif op == "sum_sha_first":
            o.check_sums(True, t)
        elif op == "sum_crc_first":
            o.check_sums(False, t)
        elif op == "big":  # larger than the default 256 KiB staging chunk: staged chunk by chunk
            o.crc_write(buf, off, 300_000 + n)
            o.sha_write(buf, off, 300_000 + n)
        elif op == "mw_two_buffers":  # equal bytes, different addresses: never bound, still right
            b2 = (ctypes.c_uint8 * n)()
            ctypes.memmove(b2, ctypes.addressof(buf) + off, n)
            o.crc_write(buf, off, n)
            o.sha_write(b2, 0, n)
    o.check_texts(rng.random() < 0.5, tag + " end")
    o.check_sums(rng.random() < 0.5, tag + " end")
    return o


@pytest.fixture
def oracle_lib(oracle):
    return oracle.lib()


def test_multiwriter_pattern_fuses_every_byte(gpu, oracle):
    """filereceiver.go's PATCH flow through FileInfo digests (32 KiB MultiWriter Writes, MarshalText
    or Sum): every pair binds at its first Write, every SHA-1 Write is served by the CRC Write's
    staged bytes, nothing is split, and the digest queue hashes each body byte ONCE."""
    h = gpu["hashing"]
    ctx = h.Context(0)
    pool = h.Pool([ctx])  # for the queue counters
    s0 = _stats(gpu)
    total = 0
    rng = random.Random(1)
    for k in range(24):
        body = rng.randbytes(rng.choice([1, 63, 64, 32768, 65536, 100_000, 1 << 20, (3 << 20) + 5]))
        fi = h.FileInfo(ctx)
        for a in range(0, len(body), 32 << 10):
            assert fi.digest.write(body[a:a + (32 << 10)]) == len(body[a:a + (32 << 10)])
        total += len(body)
        if k % 2:
            assert fi.digest.sha1.sum() == hashlib.sha1(body).digest()
            assert fi.digest.crc32.sum32() == zlib.crc32(body)
        else:
            o = oracle.Sha1()
            for a in range(0, len(body), 32 << 10):
                o.write(body[a:a + (32 << 10)])
            assert fi.digest.sha1.marshal_text().decode() == o.marshal_text()
            assert fi.digest.crc32.marshal_text().decode() == "%08x" % zlib.crc32(body)
    d = _delta(s0, _stats(gpu))
    assert d["pairs"] == 24 and d["settles"] == 0 and d["fused_bytes"] == total, d
    st = pool.stats(0)
    assert st.bytes == total, (st.bytes, total)
    pool.close()
    ctx.close()


def test_diverging_pairs_random_scripts(gpu, oracle, oracle_lib):
    """200 random scripts of Go-surface calls (MultiWriter Writes mixed with one-digest Writes,
    mutated buffers, other lengths, SHA-1 first, empty Writes, Reset / UnmarshalText of either
    member, MarshalText / Sum in either order, Writes larger than a chunk): every text and digest
    equals the oracle's; pairs were bound and split along the way."""
    gpu = dict(gpu, oracle_lib=oracle_lib)
    s0 = _stats(gpu)
    for seed in range(200):
        _script(gpu, oracle, random.Random(seed), 24, tag=f"seed {seed}")
    d = _delta(s0, _stats(gpu))
    assert d["pairs"] > 100 and d["settles"] > 50, d


@pytest.mark.parametrize("slots", ["15", "65536"])
def test_diverging_pairs_16_threads_small_queue(gpu, oracle, oracle_lib, monkeypatch, slots):
    """The same scripts from 16 threads on a context whose digest queue has 16 staging chunks and 15
    upload slots (pairs evicted and settled between their members' calls, mid-Write included) or
    65 536 (partly filled chunks of idle pairs handed over by the dispatcher), plus a pool over two
    contexts: every text and digest equals the oracle's, nothing deadlocks."""
    monkeypatch.setenv("EFES_DIGEST_STAGING_MIB", "1")
    monkeypatch.setenv("EFES_DIGEST_SLOTS", slots)
    h = gpu["hashing"]
    gpu = dict(gpu, oracle_lib=oracle_lib)
    small = h.Context(0)
    ctxs = [h.Context(0), h.Context(0)]
    pool = h.Pool(ctxs)
    errors = []

    def worker(t):
        try:
            rng = random.Random(1000 + t)
            live = []
            for s in range(6):  # several objects alive at once per thread: more pairs than slots
                kw = dict(ctx=small) if t % 2 == 0 else dict(pool=pool)
                live.append(_script(gpu, oracle, rng, 16, tag=f"thread {t} script {s}", **kw))
        except Exception as e:  # pragma: no cover - reported below
            errors.append(repr(e))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(timeout=110)
    assert not any(th.is_alive() for th in ths), "a digest call deadlocked"
    assert not errors, errors[:3]
    pool.close()
    for c in ctxs + [small]:
        c.close()


def test_member_freed_or_reset_mid_stream(gpu, oracle, oracle_lib):
    """A pair whose member is freed (the finalizer) or reset while the other is mid-stream, with an
    unconfirmed CRC Write staged: the survivor's bytes are exactly its own Writes."""
    h = gpu["hashing"]
    for case in range(4):
        o = Obj(gpu, oracle)
        buf = _buf(200_000, 77 + case)
        for a in range(0, 98304, 32768):
            o.crc_write(buf, a, 32768)
            o.sha_write(buf, a, 32768)
        o.crc_write(buf, 98304, 32768)  # staged, not yet confirmed by the SHA-1 digest
        if case == 0:  # the SHA-1 digest dies: the CRC keeps every byte it was given
            del o.sha
            assert o.crc.sum32() == o.ocrc.sum32()
        elif case == 1:  # the CRC digest dies: the SHA-1 digest never sees its unconfirmed bytes
            del o.crc
            o.sha_write(buf, 131072, 1000)
            assert o.sha.marshal_text().decode() == o.osha.marshal_text()
        elif case == 2:  # Reset of the CRC with its own Write unconfirmed
            o.crc.reset()
            o.ocrc = oracle.Crc32()
            o.sha_write(buf, 98304, 32768)
            o.crc_write(buf, 5, 99)
            o.check_sums(True, "reset crc")
        else:  # MarshalText of the CRC first with its Write unconfirmed (its bytes are its own)
            assert o.crc.marshal_text().decode() == o.ocrc.marshal_text()
            o.sha_write(buf, 98304, 32768)
            o.check_texts(True, "crc first")
        del o
    assert h  # the module stays imported while digests are freed


_MODE_CHILD = r"""
import random, sys
sys.path[:0] = [{root!r}, {tests!r}]
from oracle import oracle
oracle.build()
import efes_amd
from efes_amd import _lib, hashing
import test_gpu_pairs as T
gpu = dict(efes=efes_amd, hashing=hashing, lib=_lib.lib(), check=_lib.check, oracle_lib=oracle.lib())
s0 = hashing.pair_stats()
for seed in range(40):
    T._script(gpu, oracle, random.Random(500 + seed), 24, tag="seed %d" % seed)
s1 = hashing.pair_stats()
d = {{k: s1[k] - s0[k] for k in s0}}
assert d["pairs"] > 10 and d["settles"] > 5, d
print("ok", d)
"""


def test_diverging_pairs_64k_chunks(gpu):
    """The random scripts with EFES_DIGEST_CHUNK_KIB=64 (read when a context's digest queue is made,
    so in a child process): most Writes, not only "big", span staging chunks, so the follower stages
    the leader's scratch copy piece by piece across chunk boundaries and the pairs split mid-Write.
    Every text and digest equals the oracle's (the default 256 KiB chunk left the
    chunk-spanning paths to chance)."""
    tests = os.path.dirname(os.path.abspath(__file__))
    code = _MODE_CHILD.format(root=os.path.dirname(tests), tests=tests)
    r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, EFES_DIGEST_CHUNK_KIB="64"),
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "ok" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])


def test_large_writes_fuse_and_split_mid_write(gpu, oracle, oracle_lib):
    """Writes larger than a staging chunk (256 KiB): the MultiWriter pattern still fuses completely
    (the CRC Write waits in a scratch buffer, the SHA-1 Write stages it chunk by chunk); a buffer
    changed between the two Writes past the first chunk splits the pair mid-Write, and the SHA-1
    state is still Go's after ONE Write (MarshalText compares x with its stale bytes)."""
    h = gpu["hashing"]
    gpu = dict(gpu, oracle_lib=oracle_lib)
    ctx = h.Context(0)
    pool = h.Pool([ctx])
    buf = _buf(3_000_000, 4242)
    o = Obj(gpu, oracle, ctx)
    s0 = _stats(gpu)
    total = 0
    for off, n in ((0, 1000), (1000, (1 << 20) + 37), (1000 + (1 << 20) + 37, 700_001)):  # odd sizes: pieces
        o.crc_write(buf, off, n)                                                          # straddle blocks
        o.sha_write(buf, off, n)
        total += n
    o.check_texts(True, "large fused")
    d = _delta(s0, _stats(gpu))
    assert d["pairs"] == 1 and d["settles"] == 0 and d["fused_bytes"] == total, d
    assert pool.stats(0).bytes == total
    for k, at in enumerate((600_000, 300, 699_999)):  # past the first pieces, in the first, in the last
        off = 100_000 + 7 * k
        o.crc_write(buf, off, 700_000)
        buf[off + at] ^= 0x5A
        o.sha_write(buf, off, 700_000)
        o.check_texts(k % 2 == 0, f"split mid-Write at {at}")
        o.crc_write(buf, off + 3, 333_333)  # alone (the SHA-1 digest holds an upload after the split);
        o.sha_write(buf, off + 3, 333_333)  # the next check_texts parks both and the pair binds again
    o.check_sums(True, "end")
    assert _delta(s0, _stats(gpu))["settles"] >= 3
    del o
    pool.close()
    ctx.close()
