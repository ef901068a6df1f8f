"""ctypes binding of libefeshash.so (the C ABI declared in include/efes_hash.h).

The library is built in-tree (efes_amd/lib/libefeshash.so) by __graft_entry__.build()
or `python -m efes_amd.build`.  There is no fallback: if the library is missing or no
gfx950 device is present, calls raise.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libefeshash.so")
# Developer override for the range-checked debug build (tools/debug_checked.py); never set in production.
if os.environ.get("EFES_LIB_OVERRIDE"):
    LIB_PATH = os.environ["EFES_LIB_OVERRIDE"]

EFES_OK = 0
EFES_ERR_INVALID_DIGEST = -1
EFES_ERR_STATE = -2
EFES_ERR_HIP = -3
EFES_ERR_ARG = -4
EFES_ERR_NO_DEVICE = -5
EFES_ERR_NOMEM = -6
EFES_ERR_DEVICE_FAULT = -7

EFES_JOB_FINALIZE = 0x1
EFES_JOB_INIT = 0x2
EFES_JOB_SUM_ONLY = 0x4
EFES_HASH_SHA1, EFES_HASH_CRC32 = 0x1, 0x2
EFES_HOST_ZERO_COPY = (1 << 64) - 1
MODE_AUTO, MODE_DEEP, MODE_WIDE = 0, 1, 2
MODE_GROUP = {4: 3, 8: 4, 16: 5, 32: 6}  # grouped DEEP: lanes per job -> EFES_MODE_GROUPn
MODE_FED4 = 7  # grouped DEEP fed by producer waves on other SIMDs (EFES_MODE_FED4: 2 chains + 2 producers)
MODE_FED4E = 8  # 3 chain waves (which expand the schedule) + 1 producer per CU (EFES_MODE_FED4E)


class HostStats(ctypes.Structure):
    _fields_ = [("seconds", ctypes.c_double), ("bytes", ctypes.c_uint64), ("segments", ctypes.c_uint32),
                ("_reserved", ctypes.c_uint32)]


class PlanPart(ctypes.Structure):
    _fields_ = [("jobs", ctypes.c_uint32), ("mode", ctypes.c_int32), ("exclusive", ctypes.c_uint32),
                ("_reserved", ctypes.c_uint32)]


PLAN_MAX_PARTS = 4


class Plan(ctypes.Structure):
    """efes_plan: consecutive parts of a longest-first batch, each in its own kernel shape."""
    _fields_ = [("njobs", ctypes.c_uint32), ("nparts", ctypes.c_uint32), ("part", PlanPart * PLAN_MAX_PARTS),
                ("est_seconds", ctypes.c_double)]

    def parts(self) -> list[tuple[int, int, bool]]:
        """[(jobs, mode, exclusive)] of the parts in use."""
        return [(int(p.jobs), int(p.mode), bool(p.exclusive)) for p in self.part[: self.nparts]]


class Sha1State(ctypes.Structure):
    """efes_sha1_state == sha1.go:29-34 sha1digest (+4 pad bytes)."""
    _fields_ = [("h", ctypes.c_uint32 * 5), ("x", ctypes.c_uint8 * 64), ("_pad", ctypes.c_uint32),
                ("nx", ctypes.c_int64), ("len", ctypes.c_uint64)]


class Crc32State(ctypes.Structure):
    _fields_ = [("crc", ctypes.c_uint32)]


class Job(ctypes.Structure):
    _fields_ = [("data", ctypes.c_uint64), ("length", ctypes.c_uint64), ("sha1", ctypes.c_uint64),
                ("crc32", ctypes.c_uint64), ("sum", ctypes.c_uint64), ("status", ctypes.c_uint64),
                ("flags", ctypes.c_uint32), ("_reserved", ctypes.c_uint32)]


class QueueStats(ctypes.Structure):
    """efes_queue_stats (ABI 5): what a queue's dispatcher launched, and its upload slots."""
    _fields_ = [("launches", ctypes.c_uint64), ("jobs", ctypes.c_uint64), ("bytes", ctypes.c_uint64),
                ("free_uploads", ctypes.c_uint32), ("max_uploads", ctypes.c_uint32)]


class PairStats(ctypes.Structure):
    """efes_pair_stats (ABI 6): process-wide counters of fused CRC + SHA-1 digest pairs."""
    _fields_ = [("pairs", ctypes.c_uint64), ("fused_writes", ctypes.c_uint64), ("fused_bytes", ctypes.c_uint64),
                ("settles", ctypes.c_uint64)]


assert ctypes.sizeof(Sha1State) == 104 and ctypes.sizeof(Job) == 56 and ctypes.sizeof(QueueStats) == 32
assert ctypes.sizeof(PairStats) == 32

# numpy mirrors for building arrays of jobs / states in bulk
JOB_DTYPE = np.dtype([("data", "<u8"), ("length", "<u8"), ("sha1", "<u8"), ("crc32", "<u8"), ("sum", "<u8"),
                      ("status", "<u8"), ("flags", "<u4"), ("_reserved", "<u4")])
SHA1_STATE_DTYPE = np.dtype([("h", "<u4", (5,)), ("x", "u1", (64,)), ("_pad", "<u4"), ("nx", "<i8"),
                             ("len", "<u8")])
assert JOB_DTYPE.itemsize == 56 and SHA1_STATE_DTYPE.itemsize == 104

# Every symbol declared in include/efes_hash.h: (restype, argtypes)
_P, _S, _VP, _I, _U32, _U64 = ctypes.POINTER, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint64
SIGNATURES = {
    "efes_strerror": (ctypes.c_char_p, [_I]),
    "efes_abi_version": (_I, []),
    "efes_build_id": (ctypes.c_char_p, []),
    "efes_sha1_state_init": (None, [_P(Sha1State)]),
    "efes_device_count": (_I, []),
    "efes_ctx_create": (_I, [_I, _P(_VP)]),
    "efes_ctx_destroy": (None, [_VP]),
    "efes_ctx_device": (_I, [_VP]),
    "efes_ctx_stream": (_VP, [_VP]),
    "efes_hash_submit": (_I, [_VP, _VP, _U32, _VP]),
    "efes_hash_submit_mode": (_I, [_VP, _VP, _U32, _VP, _I]),
    "efes_auto_mode": (_I, [_VP, _U32]),
    "efes_plan_batch": (_I, [_VP, _P(_U64), _U32, _P(_U32), _P(Plan)]),
    "efes_hash_submit_plan": (_I, [_VP, _VP, _P(Plan), _VP]),
    "efes_sync": (_I, [_VP, _VP]),
    "efes_device_alloc": (_I, [_VP, _S, _P(_VP)]),
    "efes_device_free": (_I, [_VP, _VP]),
    "efes_copy_to_device": (_I, [_VP, _VP, _VP, _S, _VP]),
    "efes_copy_to_host": (_I, [_VP, _VP, _VP, _S, _VP]),
    "efes_fill_synthetic": (_I, [_VP, _VP, _S, _U64, _VP]),
    "efes_hash_host": (_I, [_VP, _VP, _U32, _U64, _P(HostStats)]),
    "efes_host_alloc": (_I, [_VP, _S, _P(_VP)]),
    "efes_host_free": (_I, [_VP, _VP]),
    "efes_queue_create": (_I, [_VP, _U64, _U32, _U32, _P(_VP)]),
    "efes_queue_destroy": (None, [_VP]),
    "efes_upload_open": (_I, [_VP, _U32, _P(Sha1State), _P(Crc32State), _P(_VP)]),
    "efes_upload_write": (_I, [_VP, _VP, _S]),
    "efes_upload_reserve": (_I, [_VP, _S, _P(_VP), _P(_S)]),
    "efes_upload_commit": (_I, [_VP, _S]),
    "efes_upload_flush": (_I, [_VP]),
    "efes_upload_state": (_I, [_VP, _P(Sha1State), _P(Crc32State)]),
    "efes_upload_sum": (_I, [_VP, _VP]),
    "efes_upload_close": (None, [_VP]),
    "efes_queue_get_stats": (_I, [_VP, _P(QueueStats)]),
    "efes_pool_create": (_I, [_P(_VP), _U32, _P(_VP)]),
    "efes_pool_destroy": (None, [_VP]),
    "efes_sha1_new_pool": (_I, [_VP, _P(_VP)]),
    "efes_sha1_new_zero_pool": (_I, [_VP, _P(_VP)]),
    "efes_crc32_new_pool": (_I, [_VP, _P(_VP)]),
    "efes_pool_stats": (_I, [_VP, _U32, _P(QueueStats)]),
    "efes_pair_stats_get": (_I, [_P(PairStats)]),
    "efes_debug_fault_after": (_I, [_VP, _U64]),
    "efes_sha1_new": (_I, [_VP, _P(_VP)]),
    "efes_sha1_new_zero": (_I, [_VP, _P(_VP)]),
    "efes_sha1_free": (None, [_VP]),
    "efes_sha1_reset": (None, [_VP]),
    "efes_sha1_size": (_I, []),
    "efes_sha1_block_size": (_I, []),
    "efes_sha1_write": (_I, [_VP, _VP, _S]),
    "efes_sha1_sum": (_I, [_VP, _VP]),
    "efes_sha1_marshal_text": (_I, [_VP, _VP]),
    "efes_sha1_unmarshal_text": (_I, [_VP, ctypes.c_char_p, _S]),
    "efes_sha1_get_state": (_I, [_VP, _P(Sha1State)]),
    "efes_sha1_set_state": (_I, [_VP, _P(Sha1State)]),
    "efes_crc32_new": (_I, [_VP, _P(_VP)]),
    "efes_crc32_free": (None, [_VP]),
    "efes_crc32_reset": (None, [_VP]),
    "efes_crc32_size": (_I, []),
    "efes_crc32_block_size": (_I, []),
    "efes_crc32_write": (_I, [_VP, _VP, _S]),
    "efes_crc32_sum32": (_I, [_VP, _P(_U32)]),
    "efes_crc32_sum": (_I, [_VP, _VP]),
    "efes_crc32_marshal_text": (_I, [_VP, _VP]),
    "efes_crc32_unmarshal_text": (_I, [_VP, ctypes.c_char_p, _S]),
    "efes_crc32_tables": (_I, [_VP, _S]),
    "efes_crc32_combine": (_U32, [_U32, _U32, _U64]),
    "efes_crc32_span": (_I, [_VP, _VP, _U64, _VP, _VP]),
    "efes_sha1_state_marshal_text": (None, [_P(Sha1State), _VP]),
    "efes_sha1_state_unmarshal_text": (_I, [_P(Sha1State), ctypes.c_char_p, _S]),
    "efes_crc32_state_marshal_text": (None, [_P(Crc32State), _VP]),
    "efes_crc32_state_unmarshal_text": (_I, [_P(Crc32State), ctypes.c_char_p, _S]),
}


class EfesError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        super().__init__(f"{what}: {strerror(code)} ({code})" if what else f"{strerror(code)} ({code})")


_lib = None


def _bind_process_hip_runtime() -> None:
    """Make the process use ONE HIP runtime.

    torch ships its own libamdhip64 (SONAME libamdhip64.so.7, ROCm 7.0); libefeshash.so
    needs libamdhip64.so.7 and would otherwise pull /opt/rocm's (7.2) through its RUNPATH.
    Two runtimes in one process do not share devices (torch then reports "No HIP GPUs").
    Importing torch first lets the dynamic linker satisfy our NEEDED entry with torch's
    already-loaded runtime.  EFES_NO_TORCH=1 skips this (pure-HIP hosts).
    """
    if os.environ.get("EFES_NO_TORCH") == "1":
        return
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def lib() -> ctypes.CDLL:
    """Load libefeshash.so (raises if it has not been built -- no fallback path exists)."""
    global _lib
    if _lib is None:
        _bind_process_hip_runtime()
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built; run __graft_entry__.build() or python -m efes_amd.build")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype, fn.argtypes = res, args
        _lib = L
    return _lib


def strerror(code: int) -> str:
    return lib().efes_strerror(code).decode()


def check(rc: int, what: str = "") -> int:
    if rc != EFES_OK:
        raise EfesError(rc, what)
    return rc
