"""Developer tool: the Sha1File read-back path (sha1file.go:9-53; write.go:69, drain.go:125) on the GPU.

Each of T threads reads its own in-memory "file" of S bytes through efes_amd.hashing.Sha1File in
32 KiB reads (one seek back and re-read half way, as a retried PATCH does), then Sums; the digests
are checked against hashlib.  Prints per-stream and aggregate MB/s for T = 1, 16, 64, 256 next to
the oracle's Sha1File (the C restatement of the Go path) on one host core.  One SHA-1 stream is a
chain: on the GPU it advances at one wavefront's issue rate (DESIGN_NOTES.md §5 "When the GPU path
pays"), so a single stream is slower than a host core and the GPU wins by concurrency.
    python tools/sha1file_rate.py [size_mib]
"""
import hashlib
import io
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from efes_amd import hashing  # noqa: E402
from oracle import oracle  # noqa: E402

size = int(sys.argv[1]) << 20 if len(sys.argv) > 1 else 16 << 20
data = np.random.default_rng(5).integers(0, 256, size, dtype=np.uint8).tobytes()
want = hashlib.sha1(data).digest()
ctx = hashing.default_context(0)


def one_stream(out, i):
    f = hashing.Sha1File(io.BytesIO(data), ctx)
    for _ in range(0, size // 2, 32 << 10):
        f.read(32 << 10)
    f.seek(size // 4)  # retry: bytes up to `calculated` are not hashed again
    while f.read(32 << 10):
        pass
    out[i] = f.sum() == want


hashing.Sha1File(io.BytesIO(b"warm"), ctx).sum()
for t in (1, 16, 64, 256):
    ok = [False] * t
    th = [threading.Thread(target=one_stream, args=(ok, i)) for i in range(t)]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    dt = time.perf_counter() - t0
    print(f"GPU Sha1File: {t:4d} streams x {size >> 20} MiB: {size / dt / 1e6:8.1f} MB/s per stream, "
          f"{t * size / dt / 1e9:7.2f} GB/s aggregate, digests ok: {all(ok)}", flush=True)
f = oracle.Sha1File(data)
t0 = time.perf_counter()
while f.read(32 << 10):
    pass
dt = time.perf_counter() - t0
print(f"CPU oracle Sha1File (1 core): {size / dt / 1e6:.1f} MB/s, digest ok: {f.sum() == want}")
