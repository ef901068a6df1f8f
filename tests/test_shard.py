"""Multi-GPU placement (efes_amd/shard.py) and the N>1 path with world_size-2 gloo on CPU.

The device work of each rank is independent (per-GPU queues, no collective), so what N>1 adds
is: every rank derives the same plan locally, every object is hashed on exactly one rank with
its chunks in order, and the job time is the max over ranks.  On CPU the per-rank hashing is
Python hashlib/zlib over the same PATCH-sized chunks (the GPU path is covered by -m gpu).
"""
import hashlib
import socket
import zlib

import numpy as np
import pytest

from efes_amd.shard import (combine_piece_crcs, gather_piece_crcs, gather_results, loads, lpt_assign,
                            max_over_ranks, piece_bounds)


def test_lpt_every_object_once_and_balanced():
    rng = np.random.default_rng(3)
    # chunksize.go-style mix: 64 KiB .. 64 MiB, log-uniform
    sizes = (64 << 10) << rng.integers(0, 11, 5000)
    for world in (1, 2, 3, 8):
        plan = lpt_assign(sizes, world)
        flat = sorted(i for q in plan for i in q)
        assert flat == list(range(len(sizes)))
        ld = loads(sizes, plan)
        # LPT bound: makespan <= 4/3 OPT, and OPT >= max(mean, largest)
        opt_lb = max(sizes.sum() / world, sizes.max())
        assert max(ld) <= 4 / 3 * opt_lb + 1
        assert plan == lpt_assign(sizes, world)  # deterministic: no communication needed


def test_lpt_edge_cases():
    assert lpt_assign([], 4) == [[], [], [], []]
    assert lpt_assign([5], 3) == [[0], [], []]
    assert lpt_assign([0, 0, 0], 2) == [[0, 2], [1]] or sorted(sum(lpt_assign([0, 0, 0], 2), [])) == [0, 1, 2]
    with pytest.raises(ValueError):
        lpt_assign([1], 0)


def test_single_process_helpers_without_dist():
    assert max_over_ranks(3.5) == 3.5
    assert gather_results({1: ("a", 2)}) == {1: ("a", 2)}


def _objects(seed=11, n=37):
    rng = np.random.default_rng(seed)
    sizes = rng.integers(0, 300_000, n)
    sizes[:3] = [0, 1, 64]
    return [rng.integers(0, 256, int(s), dtype=np.uint8).tobytes() for s in sizes]


def _hash_object(data: bytes, chunk: int):
    """One upload as PATCH chunks (write.go:126); state carried across chunks."""
    h, crc = hashlib.sha1(), 0
    for k in range(0, len(data), chunk):
        h.update(data[k:k + chunk])
        crc = zlib.crc32(data[k:k + chunk], crc)
    return h.hexdigest(), crc


def _worker(rank, world, port, q):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        objs = _objects()
        plan = lpt_assign([len(o) for o in objs], world)
        local = {i: _hash_object(objs[i], 4096) for i in plan[rank]}
        allr = gather_results(local)
        t = max_over_ranks(float(rank + 1))
        if rank == 0:
            q.put((allr, t, [len(p) for p in plan]))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_sharding_matches_single_process():
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    allr, t, counts = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    objs = _objects()
    assert allr == {i: _hash_object(o, len(o) or 1) for i, o in enumerate(objs)}  # chunking is invisible
    assert t == 2.0  # max over ranks
    assert sum(counts) == len(objs) and min(counts) > 0


def test_piece_bounds_cover_the_object():
    for length in (0, 1, 4095, 4096, 4097, 10 << 20, (10 << 20) + 3):
        for world in (1, 2, 3, 8):
            b = piece_bounds(length, world)
            assert len(b) == world and sum(n for _, n in b) == length
            assert all(a % 4096 == 0 or n == 0 for a, n in b)
            assert all(b[i][0] + b[i][1] == b[i + 1][0] or b[i + 1][1] == 0 for i in range(world - 1))


def test_combine_piece_crcs_equals_one_pass():
    """Pieces CRC'd from zero states and folded in order == crc32.go over the whole (zlib), from
    any starting state."""
    rng = np.random.default_rng(9)
    data = rng.integers(0, 256, 1_000_003, dtype=np.uint8).tobytes()
    for world in (1, 2, 5, 8):
        pieces = [(zlib.crc32(data[a:a + n]), n) for a, n in piece_bounds(len(data), world, align=64)]
        assert combine_piece_crcs(pieces) == zlib.crc32(data)
        assert combine_piece_crcs(pieces, 0xDEADBEEF) == zlib.crc32(data, 0xDEADBEEF)


def _crc_worker(rank, world, port, q):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        data = np.random.default_rng(21).integers(0, 256, 3_000_017, dtype=np.uint8).tobytes()
        a, n = piece_bounds(len(data), world)[rank]
        pieces = gather_piece_crcs(zlib.crc32(data[a:a + n]), n)  # the rank's GPU would span its piece
        q.put((rank, combine_piece_crcs(pieces)))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_object_crc_matches_single_pass():
    """One object's CRC over two ranks: each CRCs its piece, all_gather of (crc, len), fold."""
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_crc_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    data = np.random.default_rng(21).integers(0, 256, 3_000_017, dtype=np.uint8).tobytes()
    assert got == {0: zlib.crc32(data), 1: zlib.crc32(data)}
