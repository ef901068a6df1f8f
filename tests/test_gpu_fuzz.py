"""Randomised GPU parity: every kernel shape against the CPU oracle on seeded random batches.

Each batch mixes, per job: the starting state (NewSha1, a mid-stream state after random
Writes with nx != 0 and stale x bytes, Go quirk states nx == 64 / negative nx / len
inconsistent with nx, or EFES_JOB_INIT which ignores the in-state), the hashes requested
(SHA-1 + CRC-32 as filereceiver.go:208's MultiWriter, or one of them), FINALIZE or not, the
message length (biased to 64-byte block edges and the 4 KiB super-step edges of the DEEP and
grouped kernels) and a misaligned start address.  Expected values come from the oracle
(oracle/efes_oracle.c, a restatement of sha1.go / crc32.go) and zlib; everything is compared
bit for bit, the full post-Write state included.
"""
import random
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

MODES = ["deep", "wide", "group4", "group8", "group16", "group32", "fed4", "fed4e", "plan"]
EDGE_LENGTHS = [0, 1, 55, 56, 63, 64, 65, 119, 120, 127, 128, 129, 4031, 4095, 4096, 4097, 4159, 8192,
                16383, 16384, 16385, 65535, 65536, 65537, 262144 + 63]


@pytest.fixture(scope="module")
def env():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import efes_amd
    from efes_amd import hashing
    from efes_amd._lib import EFES_JOB_FINALIZE, EFES_JOB_INIT, MODE_FED4, MODE_FED4E, MODE_GROUP
    from efes_amd.batch import MODE_PLAN, DeviceBatch, fresh_states
    modes = {"deep": efes_amd.MODE_DEEP, "wide": efes_amd.MODE_WIDE, "plan": MODE_PLAN, "fed4": MODE_FED4,
             "fed4e": MODE_FED4E}
    modes.update({f"group{g}": v for g, v in MODE_GROUP.items()})
    return dict(torch=torch, ctx=hashing.default_context(0), DeviceBatch=DeviceBatch, fresh_states=fresh_states,
                modes=modes, FIN=EFES_JOB_FINALIZE, INIT=EFES_JOB_INIT)


def random_state(oracle, rng: random.Random):
    """(h, x, nx, len) of a sha1digest the reference could hold (or one of its panic states)."""
    kind = rng.random()
    s = oracle.Sha1()
    if kind < 0.25:
        pass  # NewSha1
    elif kind < 0.80:  # mid-stream after random Write calls (stale x bytes from earlier Writes)
        for _ in range(rng.randint(1, 4)):
            s.write(bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 200))))
    elif kind < 0.88:
        s.st.x[:] = bytes(rng.getrandbits(8) for _ in range(64))
        s.st.nx, s.st.len = 64, rng.choice([64, 128, 64 * rng.randint(1, 1000)])  # full pending block
    elif kind < 0.94:
        s.st.nx, s.st.len = rng.randint(1, 63), rng.getrandbits(20)  # nx inconsistent with len
    else:
        s.st.nx, s.st.len = -rng.randint(1, 9), rng.getrandbits(10)  # negative nx (Write skips it)
    return list(s.st.h), bytes(s.st.x), int(s.st.nx), int(s.st.len)


def expected(oracle, st, data: bytes, crc_in: int, sha: bool, crc: bool, fin: bool, init: bool):
    """(status, state tuple or None, crc, sum24) per the oracle for one job."""
    s = oracle.Sha1(reset=init)
    if not init:
        s.st.h[:], s.st.x[:] = st[0], st[1]
        s.st.nx, s.st.len = st[2], st[3]
    c_in = 0 if init else crc_in
    status, sum20, out_state = 0, b"\0" * 20, None
    if sha:
        rc = s.write(data)
        if rc:
            return -2, None, None, None
        out_state = (list(s.st.h), bytes(s.st.x), int(s.st.nx), int(s.st.len))
        if fin:
            src, d = s.sum()
            if src:
                status = -2
            else:
                sum20 = d
    c_out = zlib.crc32(data, c_in) if crc else None
    sum4 = c_out.to_bytes(4, "big") if crc else b"\0" * 4
    return status, out_state, c_out, (sum20 if status == 0 else b"\0" * 20) + sum4


def run_case(env, oracle, seed: int, mode: str, n: int):
    rng = random.Random(seed)
    lengths = [rng.choice(EDGE_LENGTHS) if rng.random() < 0.6 else rng.randint(0, 300000) for _ in range(n)]
    offsets, pos = [], 0
    for L in lengths:
        pos += rng.choice([0, 0, 0, 1, 2, 3, 5, 13, 16, 48, 61])
        offsets.append(pos)
        pos += L
    host = oracle.fill_synthetic(pos + 64, seed)
    buf = env["torch"].from_numpy(host).to("cuda:0")
    states = env["fresh_states"](n)
    crcs = np.zeros(n, np.uint32)
    init_states = []
    for i in range(n):
        st = random_state(oracle, rng)
        init_states.append(st)
        states[i]["h"], states[i]["x"] = st[0], np.frombuffer(st[1], np.uint8)
        states[i]["nx"], states[i]["len"] = st[2], st[3]
        crcs[i] = rng.getrandbits(32)
    hashes = [rng.choice(["both"] * 6 + ["sha", "crc"]) for _ in range(n)]
    fin = [rng.random() < 0.7 for _ in range(n)]
    init = [rng.random() < 0.15 for _ in range(n)]
    b = env["DeviceBatch"](buf.data_ptr(), offsets, lengths, states=states, crcs=crcs, ctx=env["ctx"])
    jobs = b.jobs_host
    for i in range(n):
        if hashes[i] == "crc":
            jobs[i]["sha1"] = 0
        if hashes[i] == "sha":
            jobs[i]["crc32"] = 0
        jobs[i]["flags"] = (env["FIN"] if fin[i] else 0) | (env["INIT"] if init[i] else 0)
        if not fin[i]:
            jobs[i]["sum"] = 0
    b.jobs.copy_(env["torch"].from_numpy(jobs.view(np.uint8).copy()))
    env["torch"].cuda.synchronize()
    b.run(env["modes"][mode])
    status, st, crc, sums = b.status_host(), b.states_host(), b.crc_sum(), b.sums_host()
    for i in range(n):
        data = host[offsets[i]:offsets[i] + lengths[i]].tobytes()
        sha_on, crc_on = hashes[i] != "crc", hashes[i] != "sha"
        e_status, e_state, e_crc, e_sum = expected(oracle, init_states[i], data, int(crcs[i]), sha_on, crc_on,
                                                   fin[i], init[i])
        what = (seed, mode, i, lengths[i], offsets[i] % 64, hashes[i], fin[i], init[i], init_states[i][2:])
        assert status[i] == e_status, what
        if e_state is None:  # Go panicked in Write (nx > 64): the state is not written back
            assert list(st[i]["h"]) == init_states[i][0] and int(st[i]["nx"]) == init_states[i][2], what
            continue
        if sha_on:
            assert (list(st[i]["h"]), bytes(st[i]["x"]), int(st[i]["nx"]), int(st[i]["len"])) == e_state, what
        else:
            assert bytes(st[i].tobytes()) == bytes(states[i].tobytes()), what  # untouched
        assert int(crc[i]) == (e_crc if crc_on else int(crcs[i])), what
        if fin[i]:
            assert bytes(sums[i]) == e_sum, what


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("seed", [101, 202, 303])
def test_random_batches(env, oracle, mode, seed):
    run_case(env, oracle, seed * 7 + MODES.index(mode), mode, 96)


@pytest.mark.parametrize("mode", ["deep", "group4", "fed4", "fed4e", "wide"])
def test_random_batch_more_jobs_than_simds(env, oracle, mode):
    """1100 random jobs: more than one wave per SIMD for DEEP, several waves per CU for the others."""
    run_case(env, oracle, 4242 + MODES.index(mode), mode, 1100)
