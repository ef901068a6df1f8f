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


def _rank_worker(rank, world, port, q, same_device):
    import torch.distributed as dist
    from efes_amd.shard import gather_rank_records, summarize_ranks
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        bdf = "0000:05:00.0" if same_device else f"0000:{0x05 + 0x10 * rank:02x}:00.0"
        rec = {"rank": rank, "local_rank": rank, "device": 0 if same_device else rank, "bdf": bdf,
               "GiB/s": 86.0 + rank, "kernel_ms": 46.2, "wall_s": 0.93, "spot_check": True}
        records = gather_rank_records(rec)
        if rank == 0:
            q.put((records, summarize_ranks(records, world), summarize_ranks(records, world, rehearsal=True)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("same_device", [False, True])
def test_two_rank_gloo_rank_records(same_device):
    """bench.py's N>1 line carries every rank's device (PCI address), rate, kernel
    time and spot checks, gathered to rank 0, which checks that WORLD_SIZE distinct devices did the
    work.  Two gloo ranks on CPU with stand-in records: distinct addresses pass; the same address on
    both ranks fails the check unless the run is the one-GPU rehearsal (--all-ranks-on-device0)."""
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_worker, args=(r, 2, port, q, same_device)) for r in range(2)]
    for p in procs:
        p.start()
    records, check, rehearsal = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r["rank"] for r in records] == [0, 1] and [r["GiB/s"] for r in records] == [86.0, 87.0]
    assert check["ranks_in_order"] and check["spot_checks_ok"] and check["sum_rank_GiB/s"] == 173.0
    assert check["devices_distinct"] is (not same_device) and check["ok"] is (not same_device)
    assert check["distinct_devices"] == (1 if same_device else 2)
    assert rehearsal["ok"]  # the rehearsal runs every rank on device 0 on purpose


def test_rank_summary_flags_bad_records():
    from efes_amd.shard import summarize_ranks
    good = [{"rank": r, "bdf": f"0000:0{r}:00.0", "GiB/s": 1.0, "spot_check": True} for r in range(4)]
    assert summarize_ranks(good, 4)["ok"]
    assert not summarize_ranks(good[:3], 4)["ok"]  # a rank missing
    bad = [dict(r) for r in good]
    bad[2]["spot_check"] = False
    assert not summarize_ranks(bad, 4)["ok"]
    unknown = [dict(r) for r in good]
    unknown[1]["bdf"] = None  # an address that could not be read: the check cannot say, and does not fail
    assert summarize_ranks(unknown, 4)["devices_distinct"] is None and summarize_ranks(unknown, 4)["ok"]
    dup = [dict(r) for r in unknown]
    dup[3]["bdf"] = dup[0]["bdf"]  # two ranks on one device is positive evidence: fails
    assert summarize_ranks(dup, 4)["devices_distinct"] is False and not summarize_ranks(dup, 4)["ok"]
