"""Concurrent uploads through the batching dispatcher (efes_queue / efes_upload in efes_hash.h).

`UploadQueue.open()` returns an `Upload`: the MultiWriter(CRC32, Sha1) of one upload
(filereceiver.go:208) with both states on the GPU.  `write` stages and returns (like the
io.Copy loop, filereceiver.go:209); the queue's dispatcher thread hashes the staged bytes of
all open uploads together.  `sums()` / `state()` / `marshal_text()` are the per-PATCH sync
points (filereceiver.go:99-100, 226).  Many Python threads may drive different uploads at once.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import Crc32State, Sha1State, check, lib
from .hashing import Context, default_context


class UploadQueue:
    def __init__(self, ctx: Context | None = None, chunk_bytes: int = 1 << 20, max_chunks: int = 256,
                 max_uploads: int = 255):
        self.ctx = ctx or default_context()
        h = ctypes.c_void_p()
        check(lib().efes_queue_create(self.ctx.handle, chunk_bytes, max_chunks, max_uploads, ctypes.byref(h)),
              "efes_queue_create")
        self.handle = h

    def open(self, state: Sha1State | None = None, crc: int | None = None, hashes: int = 3) -> "Upload":
        return Upload(self, state, crc, hashes)

    def close(self) -> None:
        if self.handle:
            lib().efes_queue_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):  # pragma: no cover - interpreter teardown order
        try:
            self.close()
        except Exception:
            pass


class Upload:
    """One upload's (SHA-1, CRC-32) pair, fed in the MultiWriter order of filereceiver.go:208."""

    def __init__(self, queue: UploadQueue, state: Sha1State | None = None, crc: int | None = None, hashes: int = 3):
        self.queue = queue
        h = ctypes.c_void_p()
        st = ctypes.byref(state) if state is not None else None
        cs = ctypes.byref(Crc32State(crc & 0xFFFFFFFF)) if crc is not None else None
        check(lib().efes_upload_open(queue.handle, hashes, st, cs, ctypes.byref(h)), "efes_upload_open")
        self._h = h
        self._view = None  # the last reservation's view, released when the reservation ends

    def _end_reservation(self) -> None:
        """A reservation lasts until the next call on the upload: its staging chunk may be handed to
        the dispatcher (and reused) after that, so the view is released and any later use raises."""
        if self._view is not None:
            self._view.release()
            self._view = None

    def write(self, p) -> int:
        """Write(p) of filereceiver.go:209's MultiWriter: staged (copied) before returning."""
        if isinstance(p, (bytes, bytearray)):
            ptr, n = p, len(p)  # ctypes passes the buffer address, no copy
        else:
            a = np.frombuffer(p, dtype=np.uint8) if not isinstance(p, np.ndarray) else p.view(np.uint8).reshape(-1)
            ptr, n = a.ctypes.data, a.size
        if isinstance(ptr, bytearray):
            ptr = (ctypes.c_char * n).from_buffer(ptr)
        self._end_reservation()
        check(lib().efes_upload_write(self._h, ptr, n), "Upload.write")
        return n

    def reserve(self, min_bytes: int) -> memoryview:
        """efes_upload_reserve: a writable view of >= min(min_bytes, chunk) bytes of the upload's
        pinned staging chunk (zero-copy: fill it, then commit(k))."""
        p, n = ctypes.c_void_p(), ctypes.c_size_t()
        self._end_reservation()
        check(lib().efes_upload_reserve(self._h, min_bytes, ctypes.byref(p), ctypes.byref(n)), "Upload.reserve")
        self._view = memoryview((ctypes.c_uint8 * n.value).from_address(p.value)).cast("B")
        return self._view

    def commit(self, k: int) -> None:
        """efes_upload_commit: the first k reserved bytes are one Write(p[:k]) (sha1.go:58-79)."""
        self._end_reservation()
        check(lib().efes_upload_commit(self._h, k), "Upload.commit")

    def flush(self) -> None:
        self._end_reservation()
        check(lib().efes_upload_flush(self._h), "Upload.flush")

    def state(self) -> tuple[Sha1State, int]:
        self._end_reservation()
        st, cs = Sha1State(), Crc32State()
        check(lib().efes_upload_state(self._h, ctypes.byref(st), ctypes.byref(cs)), "Upload.state")
        return st, cs.crc

    def sums(self) -> tuple[bytes, int]:
        """(SHA-1 Sum, CRC-32 Sum32) of everything written so far; the state is unchanged."""
        out = (ctypes.c_uint8 * 24)()
        self._end_reservation()
        check(lib().efes_upload_sum(self._h, out), "Upload.sums")
        b = bytes(out)
        return b[:20], int.from_bytes(b[20:], "big")

    def marshal_text(self) -> tuple[bytes, bytes]:
        """(sha1 MarshalText, crc32 MarshalText) as the .info file stores them (fileinfo.go:15-18)."""
        st, crc = self.state()
        a = ctypes.create_string_buffer(200)
        lib().efes_sha1_state_marshal_text(ctypes.byref(st), a)
        c = ctypes.create_string_buffer(8)
        lib().efes_crc32_state_marshal_text(ctypes.byref(Crc32State(crc)), c)
        return a.raw[:200], c.raw[:8]

    def close(self) -> None:
        if getattr(self, "_view", None) is not None:
            self._end_reservation()
        if getattr(self, "_h", None):
            lib().efes_upload_close(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass
