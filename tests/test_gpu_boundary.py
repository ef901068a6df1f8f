"""The Go-surface boundary under load (efes_hash.h layer 2, ABI 5), against the CPU oracle.

Go's sha1digest.Write / crc32digest.Write never fail (sha1.go:58-79, crc32.go:76-86), and
filereceiver.go creates two fresh digests per PATCH (fileinfo.go:20-27, filereceiver.go:180-182)
that only the garbage collector frees.  These tests hold that contract with a deliberately tiny
digest queue (EFES_DIGEST_STAGING_MIB=1: 16 staging chunks) with 15 upload slots (eviction) and
with 65 536 (chunk reclaim by the dispatcher):
  * 200 PATCHes, each through a NEW FileInfo that is never freed until the end;
  * more digests written-but-not-synced at once than there are slots (eviction), from 16 threads;
  * a device fault in the middle of a Write stream: Write still returns len(p), the sync points
    report the fault (MarshalText -> HTTP 500, filereceiver.go:94-96);
and the multi-GPU pool (efes_pool_*): 16 request threads' digests spread over two contexts
(standing in for two GPUs), both queues doing work, every text and Sum equal to the oracle's.
"""
import gc
import hashlib
import json
import random
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
    from efes_amd import hashing
    return dict(efes=efes_amd, hashing=hashing)


@pytest.fixture(params=["evict", "reclaim"])
def small_ctx(gpu, monkeypatch, request):
    """A fresh context whose digest queue (created at its first digest Write) has 16 staging chunks and
    either 15 upload slots (round 3's queue: a Write that finds no slot evicts an idle holder) or
    65 536 (round 4's default: more uploads than chunks, the dispatcher has idle holders hand their
    partly filled chunks over when writers wait for one)."""
    monkeypatch.setenv("EFES_DIGEST_STAGING_MIB", "1")
    monkeypatch.setenv("EFES_DIGEST_SLOTS", "15" if request.param == "evict" else "65536")
    ctx = gpu["hashing"].Context(0)
    ctx.slots = 15 if request.param == "evict" else 65536
    yield ctx
    ctx.close()


class _Counts(dict):
    def __sub__(self, o):
        return _Counts({k: self[k] - o[k] for k in self})


def pair_stats(gpu) -> _Counts:
    """efes_pair_stats_get (ABI 6): process-wide fused-pair counters."""
    return _Counts(gpu["hashing"].pair_stats())


def _payload(n: int, seed: int) -> bytes:
    return random.Random(seed).randbytes(n)


class OracleObject:
    """The reference's digests of one object (oracle = C restatement of sha1.go / crc32.go)."""

    def __init__(self, oracle):
        self.sha = oracle.Sha1()
        self.crc = oracle.Crc32()

    def write(self, p: bytes, piece: int = 32 << 10):
        """The same Write calls _patch makes (Go's stale x bytes follow the Write boundaries), in
        MultiWriter order (filereceiver.go:208): CRC32, then Sha1."""
        for k in range(0, len(p), piece):
            self.crc.write(p[k:k + piece])
            assert self.sha.write(p[k:k + piece]) == 0

    def info(self, offset: int) -> str:  # fileinfo.go:47-58
        return json.dumps({"offset": offset, "digest": {"sha1": self.sha.marshal_text(),
                                                          "crc32": self.crc.marshal_text()}},
                          separators=(",", ":")) + "\n"


def _patch(hashing, fi, body: bytes, write: int = 32 << 10):
    """saveFile's io.Copy(MultiWriter(f, CRC32, Sha1), r) in `write`-byte reads (filereceiver.go:209)."""
    for k in range(0, len(body), write):
        n = fi.digest.write(body[k:k + write])
        assert n == len(body[k:k + write])  # Write returns len(p), nil


def test_200_patches_new_fileinfo_each_never_freed(gpu, small_ctx, oracle):
    """The verdict's scenario: 20 objects x 10 PATCHes = 200 PATCHes, interleaved; every PATCH
    builds a NEW FileInfo from the saved .info text (or newFileInfo for the first), streams its
    body, then saves the .info (MarshalText) or, on the last PATCH, reads the Sums.  No FileInfo
    is freed before the end.  Every Write succeeds; every .info text and Sum equals the oracle's."""
    hashing = gpu["hashing"]
    pool1 = hashing.Pool([small_ctx])  # only to read the digest queue's counters
    p0 = pair_stats(gpu)
    objs = 20
    bodies = {o: [_payload(random.Random(o * 100 + p).choice([1, 63, 64, 65, 4097, 40000, 65536, 70001, 131072]),
                           o * 1000 + p) for p in range(10)] for o in range(objs)}
    saved = {o: None for o in range(objs)}
    expect = {o: OracleObject(oracle) for o in range(objs)}
    offset = {o: 0 for o in range(objs)}
    alive = []  # every FileInfo of every PATCH, freed only at the end (the GC never ran)
    for p in range(10):
        for o in range(objs):
            fi = (hashing.FileInfo(small_ctx) if saved[o] is None
                  else hashing.FileInfo.loads(saved[o], small_ctx))  # filereceiver.go:172-182
            alive.append(fi)
            body = bodies[o][p]
            _patch(hashing, fi, body)
            expect[o].write(body)
            offset[o] += len(body)
            fi.offset = offset[o]
            if p < 9:
                saved[o] = fi.dumps()  # SaveFileInfo (filereceiver.go:226)
                assert saved[o] == expect[o].info(offset[o]), (o, p)
            else:  # the upload is complete: the digest headers (filereceiver.go:99-100)
                data = b"".join(bodies[o])
                assert fi.digest.sha1.sum() == hashlib.sha1(data).digest()
                assert fi.digest.crc32.sum32() == zlib.crc32(data)
                assert fi.digest.sha1.marshal_text().decode() == expect[o].sha.marshal_text()
    st = pool1.stats(0)
    assert st.max_uploads == small_ctx.slots and st.free_uploads == small_ctx.slots  # all parked after their sync points
    # every PATCH's MultiWriter pair was fused: each body byte staged and hashed ONCE (two separate
    # digests hashed it twice until round 3)
    total = sum(len(b) for bs in bodies.values() for b in bs)
    assert st.jobs > 0 and st.bytes == total, (st.bytes, total)
    ps = pair_stats(gpu) - p0
    assert ps["pairs"] == 200 and ps["fused_bytes"] == total and ps["settles"] == 0, ps
    del alive
    pool1.close()


def test_more_unsynced_digests_than_slots_evict(gpu, small_ctx, oracle):
    """48 digests written to and NOT synced (as a failed saveFile abandons them to the GC) on a queue
    with 16 staging chunks: every Write succeeds -- with 15 slots the oldest idle holder is evicted
    (its staged bytes hashed, its state parked on the host), with 65 536 the idle holders' partly
    filled chunks are handed over -- and each digest, synced later, equals the oracle."""
    hashing = gpu["hashing"]
    n = 48
    digests = [hashing.Digest(small_ctx) for _ in range(n)]
    exp = [OracleObject(oracle) for _ in range(n)]
    rng = random.Random(3)
    for r in range(3):  # three rounds of Writes over all of them, never a sync point in between
        for i in range(n):
            p = _payload(rng.choice([5, 64, 1000, 33000, 65536, 65537]), r * 100 + i)
            assert digests[i].write(p) == len(p)
            exp[i].write(p, piece=len(p) or 1)
    for i in reversed(range(n)):
        assert digests[i].sha1.marshal_text().decode() == exp[i].sha.marshal_text(), i
        assert digests[i].crc32.marshal_text().decode() == exp[i].crc.marshal_text(), i
        rc, d = exp[i].sha.sum()
        assert rc == 0 and digests[i].sha1.sum() == d


def test_concurrent_threads_more_digests_than_slots(gpu, small_ctx, oracle):
    """16 request threads x 6 open objects each (96 digests on 15 slots), 32 KiB Writes in
    MultiWriter order with a sync point only every third PATCH: no Write fails or deadlocks, and
    every .info text and final Sum equals the oracle's."""
    hashing = gpu["hashing"]
    errors = []

    def worker(t):
        try:
            rng = random.Random(t)
            objs = [(hashing.FileInfo(small_ctx), OracleObject(oracle), []) for _ in range(6)]
            for p in range(6):
                for k, (fi, ex, parts) in enumerate(objs):
                    body = _payload(rng.choice([100, 32768, 50000, 65536, 98304]), t * 1000 + p * 10 + k)
                    _patch(hashing, fi, body)
                    ex.write(body)
                    parts.append(body)
                    if p % 3 == 2:
                        txt = fi.digest.to_json()
                        assert txt == {"sha1": ex.sha.marshal_text(), "crc32": ex.crc.marshal_text()}, (t, p, k)
            for fi, ex, parts in objs:
                data = b"".join(parts)
                assert fi.digest.sha1.sum() == hashlib.sha1(data).digest(), t
                assert fi.digest.crc32.sum32() == zlib.crc32(data), t
        except Exception as e:  # pragma: no cover - reported below
            errors.append(repr(e))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(timeout=100)
    assert not any(th.is_alive() for th in ths), "a digest call deadlocked"
    assert not errors, errors[:3]


def test_device_fault_is_latched_to_the_sync_point(gpu, oracle):
    """A device fault under the Writes (efes_debug_fault_after(ctx, 1): the digest queue's first
    launch reports a fault, as a faulted kernel would): every Write keeps returning len(p) -- Go's
    Write never fails -- and MarshalText / Sum report the fault (MarshalText's error -> HTTP 500).
    The queue stays faulted, as after a real device fault (a new digest there also fails at its sync
    point), while a digest on a healthy context is unaffected."""
    hashing, efes = gpu["hashing"], gpu["efes"]
    ctx = hashing.Context(0)
    ctx.debug_fault_after(1)
    d = d2 = None
    try:
        d = hashing.Digest(ctx)
        assert d.write(b"x") == 1
        for k in range(8):
            assert d.write(_payload(65536 + k, 10 + k)) == 65536 + k
        with pytest.raises(efes.EfesError) as e:
            d.sha1.marshal_text()
        assert e.value.code in (efes.EFES_ERR_DEVICE_FAULT, efes.EFES_ERR_HIP)
        with pytest.raises(efes.EfesError):
            d.sha1.sum()
        with pytest.raises(efes.EfesError):
            d.crc32.marshal_text()
        assert d.write(b"more") == 4  # still no Write error
        d.sha1.reset()  # Reset clears the object's latch; the queue is still faulted
        assert d.sha1.write(b"abc") == 3
        with pytest.raises(efes.EfesError):
            d.sha1.marshal_text()
        d2 = hashing.Digest()  # the default (healthy) context
        body = _payload(100000, 99)
        d2.write(body)
        assert d2.sha1.marshal_text().decode() == _oracle_text(oracle, body)
        assert d2.crc32.sum32() == zlib.crc32(body)
    finally:
        del d, d2
        ctx.close()


def _oracle_text(oracle, data: bytes) -> str:
    o = oracle.Sha1()
    o.write(data)
    return o.marshal_text()


def test_pool_spreads_digests_over_contexts(gpu, oracle):
    """efes_pool over two contexts (two queues, standing in for two GPUs of one process): 16 request
    threads run resumable uploads PATCH by PATCH through pooled FileInfo digests (UnmarshalText of
    the saved .info -> 32 KiB Writes in MultiWriter order -> MarshalText, Sum at the end).  Both
    contexts' digest queues launch work, and every text and digest equals the oracle's."""
    hashing = gpu["hashing"]
    ctxs = [hashing.Context(0), hashing.Context(0)]
    pool = hashing.Pool(ctxs)
    errors = []

    def worker(t):
        try:
            rng = random.Random(50 + t)
            for obj in range(3):
                ex, parts, saved, off = OracleObject(oracle), [], None, 0
                for p in range(4):
                    fi = hashing.FileInfo(pool=pool) if saved is None else hashing.FileInfo.loads(saved, pool=pool)
                    body = _payload(rng.choice([1, 4096, 65536, 200000, 1 << 20]), t * 100 + obj * 10 + p)
                    _patch(hashing, fi, body)
                    ex.write(body)
                    parts.append(body)
                    off += len(body)
                    fi.offset = off
                    if p < 3:
                        saved = fi.dumps()
                        assert saved == ex.info(off), (t, obj, p)
                    else:
                        data = b"".join(parts)
                        assert fi.digest.sha1.sum() == hashlib.sha1(data).digest()
                        assert fi.digest.crc32.sum32() == zlib.crc32(data)
        except Exception as e:  # pragma: no cover - reported below
            errors.append(repr(e))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(timeout=100)
    assert not any(th.is_alive() for th in ths)
    assert not errors, errors[:3]
    s0, s1 = pool.stats(0), pool.stats(1)
    assert s0.jobs > 0 and s1.jobs > 0, (s0.jobs, s1.jobs)
    assert s0.bytes + s1.bytes > 0
    pool.close()
    for c in ctxs:
        c.close()


def test_pool_skips_a_faulted_context(gpu, oracle):
    """a pooled digest opens its upload on the context with the most free slots -- but
    never on one whose digest queue latched a device fault (its uploads close fast and would look
    free).  Context 0's queue faults on its first launch; afterwards every new pooled digest lands
    on context 1 and equals the oracle, and context 0's queue launches nothing more."""
    hashing, efes = gpu["hashing"], gpu["efes"]
    ctxs = [hashing.Context(0), hashing.Context(0)]
    ctxs[0].debug_fault_after(1)
    pool = hashing.Pool(ctxs)
    try:
        # fault context 0: open digests until one lands there, then sync it
        d = hashing.Digest(ctx=ctxs[0])
        d.write(b"fault me")
        with pytest.raises(efes.EfesError):
            d.sha1.marshal_text()
        del d
        s0 = pool.stats(0)
        for i in range(24):
            body = _payload(70000 + i, 500 + i)
            fi = hashing.FileInfo(pool=pool)
            _patch(hashing, fi, body)
            assert fi.digest.sha1.marshal_text().decode() == _oracle_text(oracle, body), i
            assert fi.digest.crc32.sum32() == zlib.crc32(body), i
        assert pool.stats(0).launches == s0.launches  # nothing more went to the faulted queue
        assert pool.stats(1).jobs > 0
    finally:
        pool.close()
        for c in ctxs:
            c.close()


_PATIENCE_CHILD = r"""
import sys, time, hashlib, zlib
sys.path[:0] = [{root!r}]
from efes_amd import hashing
ctx = hashing.Context(0)
data = bytes(range(256)) * 400  # 102 400 bytes
a, b, c = hashing.Sha1Digest(ctx), hashing.Sha1Digest(ctx), hashing.Sha1Digest(ctx)
a.write(data)  # a and b hold the queue's two upload slots (EFES_DIGEST_SLOTS=2) ...
b.write(data[:5000])
t0 = time.perf_counter()
c.write(data)  # ... so c's Write must evict one of them, idle for a few microseconds (a SHA-1
               # digest: a CRC digest's first Write would wait in a scratch buffer for its partner)
waited = time.perf_counter() - t0
assert a.sum() == hashlib.sha1(data).digest() and b.sum() == hashlib.sha1(data[:5000]).digest()
assert c.sum() == hashlib.sha1(data).digest()
print("waited %.4f" % waited)
"""


@pytest.mark.parametrize("patience_ms", ["0", "1500"])
def test_evict_patience(gpu, patience_ms):
    """EFES_DIGEST_EVICT_MS (read when the library is loaded, so in a child process): on a queue with
    two upload slots (EFES_DIGEST_SLOTS=2, below its 16 chunks: no chunk reclaim), a third digest's
    Write evicts a holder idle for the patience -- at once with 0, after ~1.5 s with 1500 (the holders
    went idle just before it) -- and every digest still equals hashlib/zlib."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, EFES_DIGEST_EVICT_MS=patience_ms, EFES_DIGEST_SLOTS="2", EFES_DIGEST_STAGING_MIB="1")
    r = subprocess.run([sys.executable, "-c", _PATIENCE_CHILD.format(root=root)], env=env, capture_output=True,
                       text=True, timeout=110)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    waited = float(r.stdout.split("waited")[1])
    if patience_ms == "0":
        assert waited < 0.5, waited
    else:
        assert 1.3 < waited < 10, waited


_STALE_ERROR_CHILD = r"""
import ctypes, hashlib, sys, zlib
sys.path[:0] = [{root!r}]
import torch
from efes_amd import MODE_DEEP, hashing
from efes_amd.batch import DeviceBatch
hip = ctypes.CDLL("libamdhip64.so.7")  # the runtime torch loaded (one HIP runtime per process)
hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]

def poison():
    # a handled failure on this thread: HIP keeps it as the thread's last error until it is read
    p = ctypes.c_void_p()
    rc = hip.hipMalloc(ctypes.byref(p), 1 << 60)
    assert rc != 0 and hip.hipPeekAtLastError() == rc, rc

ctx = hashing.Context(0)
s = torch.cuda.Stream()
n = (8 << 20) + 3
with torch.cuda.stream(s):
    data = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    ctx.fill_synthetic(data.data_ptr(), n, 77, s.cuda_stream)
    st = torch.zeros(1, dtype=torch.int64, device="cuda:0")
    b = DeviceBatch(data.data_ptr(), [0, 1, 4096], [n - 1, 65, 1 << 20], ctx=ctx)
s.synchronize()
host = data.cpu().numpy().tobytes()
poison()
ctx.crc32_span(data.data_ptr() + 1, n - 1, st.data_ptr(), s.cuda_stream)  # raised EFES_ERR_HIP before the fix
poison()
rc = hashing.lib().efes_hash_submit_mode(ctx.handle, b.jobs.data_ptr(), b.n, s.cuda_stream, MODE_DEEP)
assert rc == 0, rc
s.synchronize()
assert int(st.item()) & 0xFFFFFFFF == zlib.crc32(host[1:])
want = [hashlib.sha1(host[o:o + k]).hexdigest() for o, k in ((0, n - 1), (1, 65), (4096, 1 << 20))]
assert (b.status_host() == 0).all() and b.sha1_hex() == want, (b.status_host(), b.sha1_hex(), want)
print("stale error ignored")
"""


def test_launches_ignore_a_stale_hip_error(gpu):
    """HIP keeps a failed call as the thread's last error until it is read.  A handled
    failure on the caller's thread -- here a hipMalloc too large to succeed; in the library, a pinned
    staging allocation retried at half size -- must not come back as the error of the next span CRC or
    job launch on that thread (every launcher clears the last error before it launches).  In a child
    process, so the poisoned thread state cannot leak into torch's own launch checks."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _STALE_ERROR_CHILD.format(root=root)], capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0 and "stale error ignored" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])


def test_python_open_devices_skips_a_failing_ordinal(gpu, oracle):
    """The Python host layer's mirror of go/hash_gpu.go pool(): open_devices() opens every ordinal below
    efes_device_count(), and with an explicit list it skips a failing ordinal in the middle and goes on;
    a Pool over the contexts that opened hashes on all of them, every text equal to the oracle's."""
    hashing = gpu["hashing"]
    n = hashing.device_count()
    assert n >= 1
    every, skipped = hashing.open_devices()
    assert [c.device for c in every] == list(range(n)) and skipped == []
    for c in every:
        c.close()
    ctxs, skipped = hashing.open_devices([0, n, 0])
    assert [c.device for c in ctxs] == [0, 0] and skipped == [(n, "invalid argument")]
    pool = hashing.Pool(ctxs)
    fis, fi = [], None
    try:
        for i in range(16):
            body = _payload(100_000 + i, 900 + i)
            fi = hashing.FileInfo(pool=pool)
            _patch(hashing, fi, body)
            fis.append((fi, body))
        for fi, body in fis:
            assert fi.digest.sha1.marshal_text().decode() == _oracle_text(oracle, body)
            assert fi.digest.crc32.sum32() == zlib.crc32(body)
        assert pool.stats(0).jobs > 0 and pool.stats(1).jobs > 0
    finally:
        fis = fi = None  # the digests go first (a pool outlives its digests, the contexts the pool)
        gc.collect()
        pool.close()
        for c in ctxs:
            c.close()
