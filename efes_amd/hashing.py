"""Python host layer over the C ABI: the reference's digest surface, GPU-backed.

Mirrors the Go types of putdotio/efes that uploads stream through:
  * ``Sha1Digest``  <- sha1digest  (sha1.go:29-120) + MarshalText/UnmarshalText (sha1_efes.go:25-64)
  * ``CRC32Digest`` <- crc32digest (crc32.go:48-93) + MarshalText/UnmarshalText (crc32_efes.go:18-40)
  * ``Sha1File``    <- Sha1File    (sha1file.go:9-53)
  * ``new_sha1`` / ``new_crc32_ieee`` <- NewSha1 (sha1.go:48) / NewCRC32IEEE (crc32.go:68)
  * ``Digest`` / ``FileInfo`` JSON  <- fileinfo.go:10-58 (the resumable `<path>.info` state)
Method names follow Python style (write/sum/marshal_text); argument meaning, return values
and error behaviour follow Go: ``write`` returns len(p); ``sum(b)`` appends the digest to b
and leaves the state untouched; ``unmarshal_text`` raises ``EfesError`` with
EFES_ERR_INVALID_DIGEST where Go returns errInvalidDigest; where the Go code would panic
the call raises ``EfesError`` with EFES_ERR_STATE.

All hashing runs on the GPU (libefeshash.so); this module only moves bytes.
"""
from __future__ import annotations

import ctypes
import io
import json
import threading

import numpy as np

from ._lib import MODE_AUTO, EfesError, PairStats, Plan, QueueStats, Sha1State, check, lib

__all__ = ["Context", "default_context", "device_count", "open_devices", "crc32_combine", "Sha1Digest", "CRC32Digest", "Sha1File", "Digest", "FileInfo",
           "new_sha1", "new_crc32_ieee", "EfesError"]


def plan_batch(lengths, ctx: "Context | None" = None) -> tuple[np.ndarray, Plan]:
    """efes_plan_batch: order[i] = index of the i-th longest job; plan = split + deep shape.

    Host-only; without a context the capacity of one MI355X (1024 SIMDs) is assumed.
    """
    lengths = np.ascontiguousarray(lengths, dtype=np.uint64)
    order = np.zeros(lengths.size, dtype=np.uint32)
    plan = Plan()
    check(lib().efes_plan_batch(ctx.handle if ctx else None, lengths.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                lengths.size, order.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), ctypes.byref(plan)),
          "efes_plan_batch")
    return order, plan


class Context:
    """efes_ctx: one GPU, its CRC tables, one stream."""

    def __init__(self, device: int = 0):
        h = ctypes.c_void_p()
        check(lib().efes_ctx_create(device, ctypes.byref(h)), "efes_ctx_create")
        self.handle = h
        self.device = device

    @property
    def stream(self) -> int:
        return lib().efes_ctx_stream(self.handle) or 0

    def submit(self, jobs_ptr: int, njobs: int, stream: int | None = None, mode: int = MODE_AUTO) -> None:
        check(lib().efes_hash_submit_mode(self.handle, jobs_ptr, njobs, stream, mode), "efes_hash_submit")

    def plan(self, lengths) -> tuple[np.ndarray, Plan]:
        """efes_plan_batch for this context's GPU: (longest-first order, plan)."""
        return plan_batch(lengths, self)

    def submit_plan(self, jobs_ptr: int, plan: Plan, stream: int | None = None) -> None:
        """efes_hash_submit_plan: a batch laid out in plan order (DEEP part on the side stream)."""
        check(lib().efes_hash_submit_plan(self.handle, jobs_ptr, ctypes.byref(plan), stream), "efes_hash_submit_plan")

    def sync(self, stream: int | None = None) -> None:
        check(lib().efes_sync(self.handle, stream), "efes_sync")

    def fill_synthetic(self, ptr: int, nbytes: int, seed: int, stream: int | None = None) -> None:
        check(lib().efes_fill_synthetic(self.handle, ptr, nbytes, seed & 0xFFFFFFFFFFFFFFFF, stream),
              "efes_fill_synthetic")

    def crc32_span(self, data_ptr: int, nbytes: int, crc_state_ptr: int, stream: int | None = None) -> None:
        """efes_crc32_span: crc32.go Write (76-86) of one long device buffer into the device CRC state
        at crc_state_ptr, segment-parallel over the whole GPU (asynchronous on `stream`)."""
        check(lib().efes_crc32_span(self.handle, data_ptr, nbytes, crc_state_ptr, stream), "efes_crc32_span")

    def debug_fault_after(self, k: int) -> None:
        """Test hook (efes_debug_fault_after): the k-th launch of this context's digest queue faults."""
        check(lib().efes_debug_fault_after(self.handle, k), "efes_debug_fault_after")

    def copy_to_host(self, dst_host: int, src_device: int, nbytes: int, stream: int | None = None) -> None:
        check(lib().efes_copy_to_host(self.handle, dst_host, src_device, nbytes, stream), "efes_copy_to_host")

    def copy_to_device(self, dst_device: int, src_host: int, nbytes: int, stream: int | None = None) -> None:
        check(lib().efes_copy_to_device(self.handle, dst_device, src_host, nbytes, stream), "efes_copy_to_device")

    def close(self) -> None:
        if self.handle:
            lib().efes_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover - interpreter teardown order
        try:
            self.close()
        except Exception:
            pass


_ctx_lock = threading.Lock()
_contexts: dict[int, Context] = {}


def default_context(device: int = 0) -> Context:
    with _ctx_lock:
        if device not in _contexts:
            _contexts[device] = Context(device)
        return _contexts[device]


class Pool:
    """efes_pool (ABI 5): digests spread over several contexts (one process over every GPU,
    server.go:130).  Each digest takes its upload slot, at every (re)open, on the context whose
    digest queue has the most free slots."""

    def __init__(self, ctxs):
        self.ctxs = list(ctxs)
        arr = (ctypes.c_void_p * len(self.ctxs))(*[c.handle.value for c in self.ctxs])
        h = ctypes.c_void_p()
        check(lib().efes_pool_create(arr, len(self.ctxs), ctypes.byref(h)), "efes_pool_create")
        self.handle = h
        self._mu = threading.Lock()
        self._live = 0  # digests made on the pool and not yet freed
        self._closing = False

    def _adopt(self) -> None:  # a digest is being made on the pool
        with self._mu:
            if self._closing or not self.handle:
                raise EfesError(-4, "pool closed")
            self._live += 1

    def _release(self) -> None:  # a digest of the pool was freed
        with self._mu:
            self._live -= 1
            last = self._closing and self._live == 0
        if last:
            self._destroy()

    def _destroy(self) -> None:
        if self.handle:
            lib().efes_pool_destroy(self.handle)
            self.handle = None

    def stats(self, i: int) -> QueueStats:
        """Counters of the digest queue of context i (efes_pool_stats)."""
        st = QueueStats()
        check(lib().efes_pool_stats(self.handle, i, ctypes.byref(st)), "efes_pool_stats")
        return st

    def close(self) -> None:
        """efes_pool_destroy -- deferred until the last digest made on the pool is freed (the C pool
        must outlive its digests: a Write of a live digest re-reads the pool's contexts)."""
        with self._mu:
            self._closing = True
            now = self._live == 0
        if now:
            self._destroy()


def device_count() -> int:
    """efes_device_count (ABI 7): HIP devices the process sees, of any architecture (0 without any)."""
    return int(lib().efes_device_count())


def open_devices(devices=None) -> tuple[list[Context], list[tuple[int, str]]]:
    """The contexts of go/hash_gpu.go's pool(): one per ordinal of `devices` (default: every ordinal
    below device_count()), skipping -- never stopping at -- the ones whose efes_ctx_create fails.
    Returns (contexts that opened, [(ordinal, reason) of each one skipped])."""
    ctxs, skipped = [], []
    for dev in (range(device_count()) if devices is None else devices):
        try:
            ctxs.append(Context(int(dev)))
        except EfesError as e:
            skipped.append((int(dev), strerror_of(e.code)))
    return ctxs, skipped


def strerror_of(code: int) -> str:
    return lib().efes_strerror(code).decode()


def pair_stats() -> dict:
    """efes_pair_stats_get (ABI 6): process-wide counters of fused CRC + SHA-1 digest pairs."""
    st = PairStats()
    check(lib().efes_pair_stats_get(ctypes.byref(st)), "efes_pair_stats_get")
    return {f: int(getattr(st, f)) for f, _ in PairStats._fields_}


def crc32_combine(crc1: int, crc2: int, len2: int) -> int:
    """CRC-32 of A||B from crc(A), crc(B), |B| (efes_crc32_combine; crc32.go is GF(2)-linear)."""
    return int(lib().efes_crc32_combine(crc1 & 0xFFFFFFFF, crc2 & 0xFFFFFFFF, len2))


def _as_bytes(p) -> bytes:
    if isinstance(p, str):
        return p.encode()
    return bytes(p)


class Sha1Digest:
    """sha1digest (sha1.go:29-34) whose compressions run on the GPU."""

    def __init__(self, ctx: Context | None = None, reset: bool = True, pool: Pool | None = None):
        h = ctypes.c_void_p()
        if pool is not None:  # the pool must outlive its digests: keep a reference, count this one
            self.ctx, self.pool = None, None
            pool._adopt()
            fn = lib().efes_sha1_new_pool if reset else lib().efes_sha1_new_zero_pool
            rc = fn(pool.handle, ctypes.byref(h))
            if rc:
                pool._release()
            check(rc, "efes_sha1_new_pool")
            self.pool = pool
        else:
            self.ctx, self.pool = ctx or default_context(), None
            fn = lib().efes_sha1_new if reset else lib().efes_sha1_new_zero
            check(fn(self.ctx.handle, ctypes.byref(h)), "efes_sha1_new")
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None):
            lib().efes_sha1_free(self._h)
            self._h = None
            if getattr(self, "pool", None) is not None:
                self.pool._release()

    def reset(self) -> None:  # sha1.go:36-44
        lib().efes_sha1_reset(self._h)

    def size(self) -> int:  # sha1.go:54
        return lib().efes_sha1_size()

    def block_size(self) -> int:  # sha1.go:56
        return lib().efes_sha1_block_size()

    def write(self, p) -> int:  # sha1.go:58-79
        b = _as_bytes(p)
        check(lib().efes_sha1_write(self._h, b, len(b)), "Sha1Digest.write")
        return len(b)

    def sum(self, b: bytes = b"") -> bytes:  # sha1.go:82-87
        out = (ctypes.c_uint8 * 20)()
        check(lib().efes_sha1_sum(self._h, out), "Sha1Digest.sum")
        return bytes(b) + bytes(out)

    def hexdigest(self) -> str:
        return self.sum().hex()

    def marshal_text(self) -> bytes:  # sha1_efes.go:25-38
        out = ctypes.create_string_buffer(200)
        check(lib().efes_sha1_marshal_text(self._h, out), "Sha1Digest.marshal_text")
        return out.raw[:200]

    def unmarshal_text(self, text) -> None:  # sha1_efes.go:40-64
        t = _as_bytes(text)
        check(lib().efes_sha1_unmarshal_text(self._h, t, len(t)), "Sha1Digest.unmarshal_text")

    def state(self) -> Sha1State:
        st = Sha1State()
        check(lib().efes_sha1_get_state(self._h, ctypes.byref(st)), "Sha1Digest.state")
        return st

    def set_state(self, st: Sha1State) -> None:
        check(lib().efes_sha1_set_state(self._h, ctypes.byref(st)), "Sha1Digest.set_state")


class CRC32Digest:
    """crc32digest (crc32.go:48-51) with the IEEE table, updated on the GPU."""

    def __init__(self, ctx: Context | None = None, pool: Pool | None = None):
        h = ctypes.c_void_p()
        if pool is not None:
            self.ctx, self.pool = None, None
            pool._adopt()
            rc = lib().efes_crc32_new_pool(pool.handle, ctypes.byref(h))
            if rc:
                pool._release()
            check(rc, "efes_crc32_new_pool")
            self.pool = pool
        else:
            self.ctx, self.pool = ctx or default_context(), None
            check(lib().efes_crc32_new(self.ctx.handle, ctypes.byref(h)), "efes_crc32_new")
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None):
            lib().efes_crc32_free(self._h)
            self._h = None
            if getattr(self, "pool", None) is not None:
                self.pool._release()

    def reset(self) -> None:  # crc32.go:74
        lib().efes_crc32_reset(self._h)

    def size(self) -> int:  # crc32.go:70
        return lib().efes_crc32_size()

    def block_size(self) -> int:  # crc32.go:72
        return lib().efes_crc32_block_size()

    def write(self, p) -> int:  # crc32.go:76-86
        b = _as_bytes(p)
        check(lib().efes_crc32_write(self._h, b, len(b)), "CRC32Digest.write")
        return len(b)

    def sum32(self) -> int:  # crc32.go:88
        v = ctypes.c_uint32()
        check(lib().efes_crc32_sum32(self._h, ctypes.byref(v)), "CRC32Digest.sum32")
        return v.value

    def sum(self, b: bytes = b"") -> bytes:  # crc32.go:90-93
        return bytes(b) + self.sum32().to_bytes(4, "big")

    def marshal_text(self) -> bytes:  # crc32_efes.go:18-24
        out = ctypes.create_string_buffer(8)
        check(lib().efes_crc32_marshal_text(self._h, out), "CRC32Digest.marshal_text")
        return out.raw[:8]

    def unmarshal_text(self, text) -> None:  # crc32_efes.go:26-40
        t = _as_bytes(text)
        check(lib().efes_crc32_unmarshal_text(self._h, t, len(t)), "CRC32Digest.unmarshal_text")


def new_sha1(ctx: Context | None = None, pool: Pool | None = None) -> Sha1Digest:  # sha1.go:48-52 NewSha1
    return Sha1Digest(ctx, pool=pool)


def new_crc32_ieee(ctx: Context | None = None, pool: Pool | None = None) -> CRC32Digest:  # crc32.go:68
    return CRC32Digest(ctx, pool=pool)


class Sha1File(io.RawIOBase):
    """sha1file.go:9-53: hashes a ReadSeeker's bytes as they are read, once each.

    ``read`` hashes only bytes beyond what was already hashed (so a retry after a seek
    back does not double-hash); reading while positioned past the hashed prefix raises
    IOError("missing data for sha1"); ``seek`` forward raises IOError("seeking forward
    is not supported") after the underlying seek, exactly as the Go code does.
    """

    def __init__(self, rs, ctx: Context | None = None):  # sha1file.go:16-21
        super().__init__()
        self.rs = rs
        self.position = 0
        self.calculated = 0
        self.digest = new_sha1(ctx)

    def readable(self) -> bool:
        return True

    def seekable(self) -> bool:
        return True

    def read(self, n: int = -1) -> bytes:  # sha1file.go:23-37
        if self.position > self.calculated:
            raise IOError("missing data for sha1")
        prev = self.position
        p = self.rs.read(n)
        self.position += len(p)
        if self.position > self.calculated:
            crop = self.calculated - prev
            c = p[crop:]
            self.digest.write(c)
            self.calculated += len(c)
        return p

    def readinto(self, b) -> int:
        p = self.read(len(b))
        b[:len(p)] = p
        return len(p)

    def seek(self, offset: int, whence: int = io.SEEK_SET) -> int:  # sha1file.go:39-49
        new_position = self.rs.seek(offset, whence)
        if self.position < new_position:
            raise IOError("seeking forward is not supported")
        self.position = new_position
        return new_position

    def tell(self) -> int:
        return self.position

    def sum(self, b: bytes = b"") -> bytes:  # sha1file.go:51-53
        return self.digest.sum(b)


class Digest:
    """fileinfo.go:15-18 `Digest{Sha1 *sha1digest "sha1"; CRC32 *crc32digest "crc32"}`."""

    def __init__(self, ctx: Context | None = None, pool: Pool | None = None):
        self.sha1 = new_sha1(ctx, pool)
        self.crc32 = new_crc32_ieee(ctx, pool)

    def write(self, p) -> int:
        """filereceiver.go:208 io.MultiWriter(f, CRC32, Sha1): CRC first, then SHA-1."""
        self.crc32.write(p)
        return self.sha1.write(p)

    def to_json(self) -> dict:
        return {"sha1": self.sha1.marshal_text().decode(), "crc32": self.crc32.marshal_text().decode()}

    def load_json(self, d: dict) -> None:
        self.sha1.unmarshal_text(d["sha1"])
        self.crc32.unmarshal_text(d["crc32"])


class FileInfo:
    """fileinfo.go:10-13 `FileInfo{Offset "offset"; Digest "digest"}` and its JSON file codec."""

    def __init__(self, ctx: Context | None = None, pool: Pool | None = None):  # fileinfo.go:20-27 newFileInfo
        self.offset = 0
        self.digest = Digest(ctx, pool)

    def dumps(self) -> str:  # fileinfo.go:47-58 json.NewEncoder(f).Encode(fi)
        return json.dumps({"offset": self.offset, "digest": self.digest.to_json()}, separators=(",", ":")) + "\n"

    @classmethod
    def loads(cls, s: str, ctx: Context | None = None, pool: Pool | None = None) -> "FileInfo":  # fileinfo.go:37-45
        d = json.loads(s)
        fi = cls(ctx, pool)
        fi.offset = int(d["offset"])
        fi.digest.load_json(d["digest"])
        return fi
