"""ctypes binding of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product package efes_amd/.  The oracle restates the
reference's Go hashing path (sha1.go, sha1_efes.go, crc32.go, crc32_efes.go,
sha1file.go); see efes_oracle.h for the pinning story.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")

OK = 0
ERR_INVALID_DIGEST = -1
ERR_PANIC = -2
ERR_SHA1FILE = -3


class Sha1State(ctypes.Structure):
    """sha1.go:29-34 sha1digest."""
    _fields_ = [("h", ctypes.c_uint32 * 5), ("x", ctypes.c_uint8 * 64),
                ("nx", ctypes.c_int64), ("len", ctypes.c_uint64)]


class Crc32State(ctypes.Structure):
    """crc32.go:48-51 crc32digest (IEEE table implied)."""
    _fields_ = [("crc", ctypes.c_uint32)]


class Sha1FileState(ctypes.Structure):
    """sha1file.go:9-14 Sha1File over an in-memory ReadSeeker."""
    _fields_ = [("data", ctypes.c_void_p), ("size", ctypes.c_int64), ("rs_pos", ctypes.c_int64),
                ("position", ctypes.c_int64), ("calculated", ctypes.c_int64), ("digest", Sha1State)]


def build() -> str:
    """Compile liboracle.so with the committed Makefile (gcc, no GPU)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P, S, U8 = ctypes.POINTER, ctypes.c_size_t, ctypes.c_uint8
        sig = {
            "oracle_sha1_reset": (None, [P(Sha1State)]),
            "oracle_sha1_block": (None, [P(Sha1State), ctypes.c_void_p, S]),
            "oracle_sha1_write": (ctypes.c_int, [P(Sha1State), ctypes.c_void_p, S]),
            "oracle_sha1_sum": (ctypes.c_int, [P(Sha1State), P(U8)]),
            "oracle_sha1_marshal_text": (None, [P(Sha1State), ctypes.c_char_p]),
            "oracle_sha1_unmarshal_text": (ctypes.c_int, [P(Sha1State), ctypes.c_char_p, S]),
            "oracle_crc32_simple_update": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_void_p, S]),
            "oracle_crc32_slicing_update": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_void_p, S]),
            "oracle_crc32_reset": (None, [P(Crc32State)]),
            "oracle_crc32_write": (None, [P(Crc32State), ctypes.c_void_p, S]),
            "oracle_crc32_sum32": (ctypes.c_uint32, [P(Crc32State)]),
            "oracle_crc32_marshal_text": (None, [P(Crc32State), ctypes.c_char_p]),
            "oracle_crc32_unmarshal_text": (ctypes.c_int, [P(Crc32State), ctypes.c_char_p, S]),
            "oracle_crc32_table": (P(ctypes.c_uint32), [ctypes.c_int]),
            "oracle_sha1file_init": (None, [P(Sha1FileState), ctypes.c_void_p, ctypes.c_int64]),
            "oracle_sha1file_read": (ctypes.c_int64, [P(Sha1FileState), ctypes.c_void_p, ctypes.c_int64]),
            "oracle_sha1file_seek": (ctypes.c_int64, [P(Sha1FileState), ctypes.c_int64, ctypes.c_int,
                                                      P(ctypes.c_int)]),
            "oracle_sha1file_sum": (ctypes.c_int, [P(Sha1FileState), P(U8)]),
            "oracle_hash_message": (None, [ctypes.c_void_p, S, S, P(U8), P(ctypes.c_uint32)]),
            "oracle_hash_many": (ctypes.c_double, [ctypes.c_void_p, S, ctypes.c_void_p, S, ctypes.c_int,
                                                   ctypes.c_void_p, ctypes.c_void_p]),
            "oracle_fill_synthetic": (None, [ctypes.c_void_p, S, ctypes.c_uint64]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype, fn.argtypes = res, args
        _lib = L
    return _lib


def _buf(data: bytes | bytearray | np.ndarray):
    """Return (pointer, length, keepalive) for bytes-like input."""
    if isinstance(data, np.ndarray):
        a = np.ascontiguousarray(data, dtype=np.uint8)
        return a.ctypes.data, a.nbytes, a
    b = (ctypes.c_uint8 * max(len(data), 1)).from_buffer_copy(bytes(data) or b"\0")
    return ctypes.addressof(b), len(data), b


class Sha1:
    """Python face of oracle_sha1 (sha1.go:29-120, sha1_efes.go:25-64)."""

    def __init__(self, reset: bool = True):
        self.st = Sha1State()
        if reset:
            lib().oracle_sha1_reset(ctypes.byref(self.st))

    def write(self, data) -> int:
        p, n, keep = _buf(data)
        return lib().oracle_sha1_write(ctypes.byref(self.st), p, n)

    def sum(self) -> tuple[int, bytes]:
        out = (ctypes.c_uint8 * 20)()
        rc = lib().oracle_sha1_sum(ctypes.byref(self.st), out)
        return rc, bytes(out)

    def hexdigest(self) -> str:
        rc, d = self.sum()
        if rc:
            raise RuntimeError(f"oracle sha1 sum failed rc={rc}")
        return d.hex()

    def marshal_text(self) -> str:
        out = ctypes.create_string_buffer(201)
        lib().oracle_sha1_marshal_text(ctypes.byref(self.st), out)
        return out.raw[:200].decode()

    def unmarshal_text(self, text: str | bytes) -> int:
        t = text.encode() if isinstance(text, str) else bytes(text)
        return lib().oracle_sha1_unmarshal_text(ctypes.byref(self.st), t, len(t))

    @property
    def h(self):
        return list(self.st.h)

    @property
    def x(self) -> bytes:
        return bytes(self.st.x)

    @property
    def nx(self) -> int:
        return self.st.nx

    @property
    def length(self) -> int:
        return self.st.len


class Crc32:
    """Python face of oracle_crc32 (crc32.go:48-93, crc32_efes.go:18-40)."""

    def __init__(self):
        self.st = Crc32State(0)

    def write(self, data) -> None:
        p, n, keep = _buf(data)
        lib().oracle_crc32_write(ctypes.byref(self.st), p, n)

    def sum32(self) -> int:
        return lib().oracle_crc32_sum32(ctypes.byref(self.st))

    def marshal_text(self) -> str:
        out = ctypes.create_string_buffer(9)
        lib().oracle_crc32_marshal_text(ctypes.byref(self.st), out)
        return out.raw[:8].decode()

    def unmarshal_text(self, text: str | bytes) -> int:
        t = text.encode() if isinstance(text, str) else bytes(text)
        return lib().oracle_crc32_unmarshal_text(ctypes.byref(self.st), t, len(t))


class Sha1File:
    """Python face of oracle_sha1file (sha1file.go:9-53) over bytes."""

    def __init__(self, data: bytes):
        self._keep = (ctypes.c_uint8 * max(len(data), 1)).from_buffer_copy(data or b"\0")
        self.st = Sha1FileState()
        lib().oracle_sha1file_init(ctypes.byref(self.st), ctypes.addressof(self._keep), len(data))

    def read(self, n: int) -> bytes:
        buf = (ctypes.c_uint8 * max(n, 1))()
        got = lib().oracle_sha1file_read(ctypes.byref(self.st), buf, n)
        if got < 0:
            raise IOError("missing data for sha1")
        return bytes(buf)[:got]

    def seek(self, offset: int, whence: int = 0) -> int:
        err = ctypes.c_int(0)
        pos = lib().oracle_sha1file_seek(ctypes.byref(self.st), offset, whence, ctypes.byref(err))
        if err.value == 1:
            raise IOError("negative position")
        if err.value == 2:
            raise IOError("seeking forward is not supported")
        return pos

    def sum(self) -> bytes:
        out = (ctypes.c_uint8 * 20)()
        lib().oracle_sha1file_sum(ctypes.byref(self.st), out)
        return bytes(out)


def hash_message(data, copy_buf: int = 32 * 1024) -> tuple[str, int]:
    """filereceiver.go:208-209 MultiWriter(file, CRC32, Sha1) over one message -> (sha1 hex, crc32)."""
    p, n, keep = _buf(data)
    out = (ctypes.c_uint8 * 20)()
    crc = ctypes.c_uint32(0)
    lib().oracle_hash_message(p, n, copy_buf, out, ctypes.byref(crc))
    return bytes(out).hex(), crc.value


def hash_many(buf: np.ndarray, stride: int, lens: np.ndarray, nthreads: int):
    """Hash len(lens) messages at buf[i*stride:] on nthreads threads -> (seconds, sha1[n,20], crc[n])."""
    lens = np.ascontiguousarray(lens, dtype=np.uint64)
    n = lens.size
    sha = np.zeros((n, 20), dtype=np.uint8)
    crc = np.zeros(n, dtype=np.uint32)
    secs = lib().oracle_hash_many(buf.ctypes.data, stride, lens.ctypes.data, n, nthreads,
                                  sha.ctypes.data, crc.ctypes.data)
    return secs, sha, crc


def fill_synthetic(n: int, seed: int) -> np.ndarray:
    """Host copy of the synthetic byte stream (same generator as efes_fill_synthetic on device)."""
    a = np.empty(n, dtype=np.uint8)
    if n:
        lib().oracle_fill_synthetic(a.ctypes.data, n, seed & 0xFFFFFFFFFFFFFFFF)
    return a


def crc32_table(k: int) -> np.ndarray:
    p = lib().oracle_crc32_table(k)
    return np.ctypeslib.as_array(p, shape=(256,)).copy()
