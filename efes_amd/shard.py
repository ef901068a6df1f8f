"""Multi-GPU placement of independent uploads: per-GPU work queues, no collectives on the data path.

Objects (uploads) are independent units: each one's chunks must be hashed in order on ONE
device because the SHA-1 state chains from chunk to chunk (filereceiver.go:182-226 resumes
the `.info` state per PATCH).  So the unit of placement is the object, and a rank's queue is
just a list of objects.  Placement is longest-processing-time-first (LPT) by byte count,
which bounds the makespan by 4/3 of optimal and matters for config 4's 64 KiB..64 MiB mix
(SURVEY.md §8(d)), where one long object sets the tail.

The only cross-rank communication is for measurement (max-over-ranks wall time) and, in the
tests, gathering digests to compare against a single-process run.
"""
from __future__ import annotations

import heapq
import os

import numpy as np


def lpt_assign(sizes, world: int) -> list[list[int]]:
    """Object indices per rank: largest first onto the least-loaded rank (ties -> lower rank).

    Deterministic, so every rank computes the same plan locally without communicating.
    """
    if world < 1:
        raise ValueError("world must be >= 1")
    sizes = np.asarray(sizes, dtype=np.int64)
    order = np.argsort(-sizes, kind="stable")
    heap = [(0, r) for r in range(world)]
    out: list[list[int]] = [[] for _ in range(world)]
    for i in order:
        load, r = heapq.heappop(heap)
        out[r].append(int(i))
        heapq.heappush(heap, (load + int(sizes[i]), r))
    for q in out:
        q.sort()  # stable submission order within a rank
    return out


def loads(sizes, plan) -> list[int]:
    sizes = np.asarray(sizes, dtype=np.int64)
    return [int(sizes[q].sum()) if q else 0 for q in plan]


def env_rank() -> tuple[int, int, int]:
    """(rank, local_rank, world_size) from the torch.distributed.run environment (defaults 0, 0, 1)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def max_over_ranks(value: float, device=None) -> float:
    """Max of a per-rank scalar (the job's wall time is the slowest rank's)."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_results(local: dict[int, tuple[str, int]]) -> dict[int, tuple[str, int]]:
    """Union of every rank's {object index: (sha1 hex, crc32)} (tests / verification only)."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return dict(local)
    parts: list = [None] * dist.get_world_size()
    dist.all_gather_object(parts, local)
    out: dict[int, tuple[str, int]] = {}
    for p in parts:
        dup = set(out) & set(p)
        if dup:
            raise RuntimeError(f"objects hashed on two ranks: {sorted(dup)[:5]}")
        out.update(p)
    return out


# ---- one object's CRC-32 over several GPUs ------------------------
# SHA-1 of an object cannot be split (one chain), but CRC-32 can: rank r spans piece r of the
# object from a zero state (efes_crc32_span on its GPU), the ranks exchange their 4-byte CRCs and
# piece lengths (one all_gather: the only data-path collective, 16 bytes per rank), and every rank
# folds them in piece order with the GF(2) combine of crc32.go's linearity (efes_crc32_combine).


def piece_bounds(length: int, world: int, align: int = 4096) -> list[tuple[int, int]]:
    """[(offset, length)] of `world` contiguous pieces covering [0, length), piece starts on
    `align`-byte boundaries (the last piece takes the remainder; pieces may be empty)."""
    if world < 1:
        raise ValueError("world must be >= 1")
    per = -(-length // world)
    per = -(-per // align) * align if per else 0
    out = []
    for r in range(world):
        a = min(length, r * per)
        out.append((a, min(length, a + per) - a))
    return out


def combine_piece_crcs(pieces, crc_in: int = 0) -> int:
    """crc32.go Write of the concatenated pieces into a state holding crc_in, from each piece's
    CRC from a zero state: [(crc, length)] in object order."""
    from efes_amd.hashing import crc32_combine

    crc = crc_in & 0xFFFFFFFF
    for c, n in pieces:
        crc = crc32_combine(crc, int(c), int(n))
    return crc


def gather_piece_crcs(crc: int, length: int, device=None) -> list[tuple[int, int]]:
    """Every rank's (crc, length), in rank order (all_gather of 16 bytes per rank)."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [(crc & 0xFFFFFFFF, length)]
    mine = torch.tensor([crc & 0xFFFFFFFF, length], dtype=torch.int64, device=device)
    parts = [torch.empty_like(mine) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, mine)
    return [(int(p[0].item()), int(p[1].item())) for p in parts]


# ---- per-rank records of a multi-GPU bench (bench.py) -------------------------------
# A weak-scaling line is only evidence of N GPUs if it shows that N distinct devices did the work:
# every rank reports its device's PCI address, its own rate, its kernel time and spot checks of its
# digests, and rank 0 checks that the addresses are distinct.


def gather_rank_records(record: dict) -> list[dict]:
    """Every rank's record, in rank order (all_gather_object; measurement only, after the timed region)."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [dict(record)]
    parts: list = [None] * dist.get_world_size()
    dist.all_gather_object(parts, dict(record))
    return parts


def summarize_ranks(records: list[dict], world: int, rehearsal: bool = False) -> dict:
    """The checks rank 0 makes on the gathered records: one record per rank, in order; no two ranks on
    one PCI address (unless `rehearsal`: every rank on device 0 of a one-GPU box; an address that could
    not be read leaves `devices_distinct` None, which does not fail the run); every rank's spot checks
    true.  `ok` is the conjunction; the rates are summed for comparison with `value`."""
    ranks = [r.get("rank") for r in records]
    bdfs = [r.get("bdf") for r in records]
    known = [b for b in bdfs if b]
    # True: every rank's address known and all different; False: two ranks on one address (positive
    # evidence of a broken placement); None: an address could not be read, so the check cannot say
    distinct = False if len(set(known)) < len(known) else (True if len(known) == world else None)
    out = {
        "world": world,
        "ranks_in_order": ranks == list(range(world)),
        "distinct_devices": len(set(known)),
        "devices_distinct": distinct,
        "rehearsal_one_device": bool(rehearsal),
        "spot_checks_ok": all(bool(r.get("spot_check")) for r in records),
        "sum_rank_GiB/s": round(sum(float(r.get("GiB/s", 0.0)) for r in records), 3),
    }
    out["ok"] = out["ranks_in_order"] and out["spot_checks_ok"] and (distinct is not False or bool(rehearsal))
    return out
