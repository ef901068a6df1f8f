"""Device-resident batches of independent jobs (layer 1 of include/efes_hash.h).

A batch is N independent `Write(p)` (+ Sum) jobs over messages that already live in
device memory -- the shape of many concurrent uploads (filereceiver.go:208-209, one
request goroutine per upload).  Device buffers are torch tensors (plumbing only); the
hashing is libefeshash.so.
"""
from __future__ import annotations

import numpy as np

from ._lib import (EFES_JOB_FINALIZE, EFES_JOB_INIT, EFES_JOB_SUM_ONLY, JOB_DTYPE, MODE_AUTO, MODE_DEEP, MODE_FED4,
                   MODE_FED4E, MODE_GROUP, MODE_WIDE, PLAN_MAX_PARTS, SHA1_STATE_DTYPE, Plan, PlanPart)
from .hashing import Context, default_context

MODE_PLAN = -1  # run(): efes_plan_batch + efes_hash_submit_plan instead of one fixed kernel shape

# lanes per job -> kernel shape, in forced_plan's spec (64 = DEEP, 0 = WIDE, 1 = FED4, 2 = FED4E)
_SPEC_MODES = {64: MODE_DEEP, 0: MODE_WIDE, 1: MODE_FED4, 2: MODE_FED4E, **MODE_GROUP}


def forced_plan(n: int, spec: str) -> Plan:
    """A caller-built efes_plan (efes_hash.h lets a caller place its own parts) for n longest-first
    jobs: "<lanes>:<jobs>[x],..." -- lanes 64 = DEEP, 0 = WIDE, 1 = FED4, 2 = FED4E (both always own
    their CUs), 4/8/16/32 = GROUPn; x = exclusive (CUs of its own) -- in order, the jobs beyond the
    listed parts WIDE.  Raises ValueError for an unknown shape or more than PLAN_MAX_PARTS parts."""
    parts, used = [], 0
    for item in filter(None, spec.split(",")):
        lanes, _, jobs = item.partition(":")
        excl = jobs.endswith("x")
        if int(lanes) not in _SPEC_MODES:
            raise ValueError(f"unknown shape {lanes!r}")
        take = min(int(jobs.rstrip("x")), n - used)
        if take:
            parts.append((take, _SPEC_MODES[int(lanes)], excl))
        used += take
    if used < n:
        parts.append((n - used, MODE_WIDE, False))
    if len(parts) > PLAN_MAX_PARTS:
        raise ValueError(f"{len(parts)} parts > {PLAN_MAX_PARTS}")
    plan = Plan()
    plan.njobs, plan.nparts = n, len(parts)
    for i, (j, m, x) in enumerate(parts):
        plan.part[i] = PlanPart(j, m, 1 if x else 0, 0)
    return plan

IV = np.array([0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476, 0xC3D2E1F0], dtype=np.uint32)


def fresh_states(n: int) -> np.ndarray:
    """n states equal to NewSha1() (sha1.go:48-52)."""
    st = np.zeros(n, dtype=SHA1_STATE_DTYPE)
    st["h"][:] = IV
    return st


class DeviceBatch:
    """Jobs j = 0..N-1: Write(data[offsets[j] : offsets[j]+lengths[j]]) into state j (+ Sum).

    Kernels run on torch's current stream.  When that is the null stream (handle 0, which
    efes_hash.h maps to the context's own non-blocking stream), submit() orders the context
    stream after the work torch queued so far and torch's stream after the launch, so
    reset() / result reads on torch's stream stay ordered with the kernels either way.
    """

    def __init__(self, data_ptr: int, offsets, lengths, *, sha1: bool = True, crc32: bool = True,
                 finalize: bool = True, fresh: bool = False, states: np.ndarray | None = None, crcs: np.ndarray | None = None,
                 ctx: Context | None = None, device: str = "cuda:0", sum_only: bool = False):
        import torch

        self.ctx = ctx or default_context(int(device.split(":")[1]) if ":" in device else 0)
        self.torch = torch
        self.device = device
        offsets = np.asarray(offsets, dtype=np.uint64)
        lengths = np.asarray(lengths, dtype=np.uint64)
        n = self.n = int(offsets.size)
        assert lengths.size == n
        self.init_states = fresh_states(n) if states is None else np.array(states, dtype=SHA1_STATE_DTYPE)
        self.init_crcs = np.zeros(n, np.uint32) if crcs is None else np.asarray(crcs, dtype=np.uint32)
        self._init_states_dev = torch.from_numpy(self.init_states.view(np.uint8).copy()).to(device)
        self._init_crcs_dev = torch.from_numpy(self.init_crcs.view(np.uint8).copy()).to(device)
        self.states = self._init_states_dev.clone()
        self.crcs = self._init_crcs_dev.clone()
        self.sums = torch.zeros(max(n, 1) * 24, dtype=torch.uint8, device=device)
        self.status = torch.full((max(n, 1),), -99, dtype=torch.int32, device=device)
        jobs = np.zeros(n, dtype=JOB_DTYPE)
        jobs["data"] = np.uint64(data_ptr) + offsets
        jobs["length"] = lengths
        if sha1:
            jobs["sha1"] = np.uint64(self.states.data_ptr()) + np.arange(n, dtype=np.uint64) * np.uint64(104)
        if crc32:
            jobs["crc32"] = np.uint64(self.crcs.data_ptr()) + np.arange(n, dtype=np.uint64) * np.uint64(4)
        if finalize:
            jobs["sum"] = np.uint64(self.sums.data_ptr()) + np.arange(n, dtype=np.uint64) * np.uint64(24)
            jobs["flags"] |= EFES_JOB_FINALIZE
        if fresh:  # new chunks: start from NewSha1()/NewCRC32IEEE(), in-states are not read
            jobs["flags"] |= EFES_JOB_INIT
        if sum_only:  # Sum of the in-states on a copy (sha1.go:82-87): states are not written
            assert finalize and not lengths.any(), "sum_only jobs are zero-length FINALIZE jobs"
            jobs["flags"] |= EFES_JOB_SUM_ONLY
        jobs["status"] = np.uint64(self.status.data_ptr()) + np.arange(n, dtype=np.uint64) * np.uint64(4)
        self.jobs_host = jobs
        self.jobs = torch.from_numpy(jobs.view(np.uint8).copy()).to(device)
        torch.cuda.synchronize(device)

    def variant(self, *, fresh: bool, finalize: bool) -> "DeviceBatch":
        """The same jobs over the same data, states, sums and status with other flags: one segment
        of a resumed Write sequence (EFES_JOB_INIT on the first segment, EFES_JOB_FINALIZE on the
        last; the states stay in HBM between them, filereceiver.go:182-226)."""
        import copy

        v = copy.copy(self)
        jobs = self.jobs_host.copy()
        jobs["flags"] &= np.uint32(~(EFES_JOB_INIT | EFES_JOB_FINALIZE) & 0xFFFFFFFF)
        if fresh:
            jobs["flags"] |= EFES_JOB_INIT
        if finalize:
            assert int(self.jobs_host["sum"][0]) != 0, "a finalizing variant needs a batch made with finalize=True"
            jobs["flags"] |= EFES_JOB_FINALIZE
        v.jobs_host = jobs
        v.jobs = self.torch.from_numpy(jobs.view(np.uint8).copy()).to(self.device)
        if hasattr(v, "plan"):
            del v.plan
        self.torch.cuda.synchronize(self.device)
        return v

    def stream(self) -> int:
        return self.torch.cuda.current_stream(self.device).cuda_stream

    def reset(self) -> None:
        """Restore the initial states (async, on torch's current stream)."""
        self.states.copy_(self._init_states_dev)
        self.crcs.copy_(self._init_crcs_dev)

    def submit(self, mode: int = MODE_AUTO) -> None:
        """Enqueue all jobs, ordered after the work on torch's current stream (data writes,
        reset()) and before the work queued there afterwards (result copies)."""
        cur = self.torch.cuda.current_stream(self.device)
        if cur.cuda_stream:
            self._launch(mode, cur.cuda_stream)
            return
        # Null stream: the library launches on the context's non-blocking stream, which the
        # null stream does not order against; join the two both ways with events.
        ctx_stream = self.torch.cuda.ExternalStream(self.ctx.stream, device=self.device)
        ctx_stream.wait_stream(cur)
        self._launch(mode, ctx_stream.cuda_stream)
        cur.wait_stream(ctx_stream)

    def _launch(self, mode: int, stream: int) -> None:
        if mode == MODE_PLAN:
            if not hasattr(self, "plan"):
                self.make_plan()
            self.ctx.submit_plan(self.jobs_planned.data_ptr(), self.plan, stream)
        else:
            self.ctx.submit(self.jobs.data_ptr(), self.n, stream, mode)

    def run(self, mode: int = MODE_AUTO) -> None:
        self.submit(mode)
        self.torch.cuda.synchronize(self.device)

    def make_plan(self, force: str | None = None) -> None:
        """efes_plan_batch over the job lengths; keeps a longest-first copy of the job array.  `force`
        replaces the planner's parts by caller-built ones (forced_plan) over the same order."""
        order, self.plan = self.ctx.plan(self.jobs_host["length"])
        if force is not None:
            self.plan = forced_plan(self.n, force)
        self.jobs_planned = self.torch.from_numpy(self.jobs_host[order].view(np.uint8).copy()).to(self.device)
        self.torch.cuda.synchronize(self.device)

    def submit_planned(self) -> None:
        """The planned launch (DEEP/grouped part concurrent with the WIDE part), ordered like submit()."""
        self.submit(MODE_PLAN)

    # ---- results (host copies)
    def status_host(self) -> np.ndarray:
        return self.status.cpu().numpy()[: self.n]

    def sums_host(self) -> np.ndarray:
        return self.sums.cpu().numpy()[: self.n * 24].reshape(self.n, 24)

    def sha1_hex(self) -> list[str]:
        s = self.sums_host()
        return [bytes(r[:20]).hex() for r in s]

    def crc_sum(self) -> np.ndarray:
        return self.crcs.cpu().numpy().view(np.uint32)[: self.n]

    def states_host(self) -> np.ndarray:
        return self.states.cpu().numpy().view(SHA1_STATE_DTYPE)[: self.n]


class PinnedHostBuffer:
    """Pinned host memory from efes_host_alloc (a socket-buffer pool registered for DMA)."""

    def __init__(self, nbytes: int, ctx: Context | None = None):
        import ctypes

        from ._lib import check, lib

        self.ctx = ctx or default_context()
        p = ctypes.c_void_p()
        check(lib().efes_host_alloc(self.ctx.handle, nbytes, ctypes.byref(p)), "efes_host_alloc")
        self.ptr = p.value
        self.nbytes = nbytes
        self.array = np.ctypeslib.as_array((ctypes.c_uint8 * max(nbytes, 1)).from_address(self.ptr))[:nbytes]

    def free(self) -> None:
        from ._lib import lib

        if self.ptr:
            self.array = None
            lib().efes_host_free(self.ctx.handle, self.ptr)
            self.ptr = None

    def __del__(self):  # pragma: no cover - interpreter teardown order
        try:
            self.free()
        except Exception:
            pass


class HostBatch:
    """Jobs whose bytes, states and sums live in HOST memory (efes_hash_host).

    Message j = host bytes [data_ptr + offsets[j], + lengths[j]); each is copied to HBM in
    `segment_bytes` pieces on a copy stream while the previous piece hashes (the per-PATCH
    resume of filereceiver.go:182-226, with the state kept on the device).
    """

    def __init__(self, data_ptr: int, offsets, lengths, *, sha1: bool = True, crc32: bool = True,
                 finalize: bool = True, fresh: bool = True, states: np.ndarray | None = None,
                 crcs: np.ndarray | None = None, ctx: Context | None = None):
        self.ctx = ctx or default_context()
        offsets = np.asarray(offsets, dtype=np.uint64)
        lengths = np.asarray(lengths, dtype=np.uint64)
        n = self.n = int(offsets.size)
        self.states = fresh_states(n) if states is None else np.array(states, dtype=SHA1_STATE_DTYPE)
        self.crcs = np.zeros(n, np.uint32) if crcs is None else np.array(crcs, dtype=np.uint32)
        self.sums = np.zeros((max(n, 1), 24), np.uint8)
        self.status = np.full(max(n, 1), -99, np.int32)
        jobs = np.zeros(n, dtype=JOB_DTYPE)
        jobs["data"] = np.uint64(data_ptr) + offsets
        jobs["length"] = lengths
        idx = np.arange(n, dtype=np.uint64)
        if sha1:
            jobs["sha1"] = np.uint64(self.states.ctypes.data) + idx * np.uint64(SHA1_STATE_DTYPE.itemsize)
        if crc32:
            jobs["crc32"] = np.uint64(self.crcs.ctypes.data) + idx * np.uint64(4)
        if finalize:
            jobs["sum"] = np.uint64(self.sums.ctypes.data) + idx * np.uint64(24)
            jobs["flags"] |= EFES_JOB_FINALIZE
        if fresh:
            jobs["flags"] |= EFES_JOB_INIT
        jobs["status"] = np.uint64(self.status.ctypes.data) + idx * np.uint64(4)
        self.jobs = jobs

    def run(self, segment_bytes: int = 1 << 20):
        """Returns efes_host_stats (seconds, bytes, segments) of the copy+hash pipeline."""
        import ctypes

        from ._lib import HostStats, check, lib

        st = HostStats()
        check(lib().efes_hash_host(self.ctx.handle, self.jobs.ctypes.data, self.n, segment_bytes,
                                   ctypes.byref(st)), "efes_hash_host")
        return st

    def sha1_hex(self) -> list[str]:
        return [bytes(r[:20]).hex() for r in self.sums[: self.n]]

    def crc_sum(self) -> np.ndarray:
        return self.crcs[: self.n]
