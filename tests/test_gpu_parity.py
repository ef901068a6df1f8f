"""GPU parity: the gfx950 kernels (through the C ABI) against the CPU oracle and golden vectors.

Bit-exact on everything: SHA-1 digests, CRC-32 values, and the full post-Write state
(h, all 64 bytes of x including the stale tail, nx, len) that MarshalText serialises.
"""
import hashlib
import io
import random
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import efes_amd
    from efes_amd import hashing
    from efes_amd.batch import DeviceBatch, fresh_states
    ctx = hashing.default_context(0)
    return dict(torch=torch, efes=efes_amd, hashing=hashing, DeviceBatch=DeviceBatch, fresh_states=fresh_states,
                ctx=ctx)


MODE_IDS = ["deep", "wide", "group4", "group8", "group16", "group32", "fed4", "fed4e", "plan"]


def _modes(env):
    from efes_amd._lib import MODE_GROUP
    from efes_amd.batch import MODE_PLAN
    from efes_amd._lib import MODE_FED4, MODE_FED4E
    m = {"deep": env["efes"].MODE_DEEP, "wide": env["efes"].MODE_WIDE, "plan": MODE_PLAN, "fed4": MODE_FED4,
         "fed4e": MODE_FED4E}
    m.update({f"group{g}": v for g, v in MODE_GROUP.items()})
    return m


def device_buffer(env, host: np.ndarray):
    t = env["torch"].from_numpy(host).to("cuda:0")
    env["torch"].cuda.synchronize()
    return t


def oracle_expect(oracle, state_row, data: bytes, crc_in: int, finalize: bool = True, writes: int = 0):
    """Expected (status, state dict, crc, sha1 sum bytes|None) of one job per the CPU oracle.

    writes > 0: the data arrives as Write calls of that many bytes (the last one shorter)."""
    s = oracle.Sha1(reset=False)
    s.st.h[:] = [int(v) for v in state_row["h"]]
    s.st.x[:] = bytes(state_row["x"])
    s.st.nx = int(state_row["nx"])
    s.st.len = int(state_row["len"])
    crc = zlib.crc32(data, crc_in)
    if writes:
        rc = 0
        for k in range(0, max(len(data), 1), writes):
            rc = rc or s.write(data[k:k + writes])
    else:
        rc = s.write(data)
    if rc:
        return -2, None, None, None
    src, digest = s.sum()
    if not finalize:
        src = 0
    return (0 if src == 0 else -2), dict(h=list(s.st.h), x=bytes(s.st.x), nx=s.st.nx, len=s.st.len), crc, \
        (digest if src == 0 else None)


def check_batch(b, oracle, datas, states, crcs, finalize=True, what=""):
    status = b.status_host()
    st = b.states_host()
    crc = b.crc_sum()
    sums = b.sums_host()
    for i, data in enumerate(datas):
        e_status, e_state, e_crc, e_sum = oracle_expect(oracle, states[i], data, int(crcs[i]), finalize)
        assert status[i] == e_status, (what, i, len(data), status[i], e_status)
        if e_state is None:
            # Go panicked inside Write: nothing written back
            assert list(st[i]["h"]) == list(states[i]["h"]) and st[i]["nx"] == states[i]["nx"], (what, i)
            continue
        assert list(st[i]["h"]) == e_state["h"], (what, i, len(data))
        assert bytes(st[i]["x"]) == e_state["x"], (what, i, len(data))
        assert int(st[i]["nx"]) == e_state["nx"] and int(st[i]["len"]) == e_state["len"], (what, i)
        assert int(crc[i]) == e_crc, (what, i, len(data))
        if finalize and e_sum is not None:
            assert bytes(sums[i][:20]) == e_sum, (what, i, len(data))
            assert bytes(sums[i][20:]) == e_crc.to_bytes(4, "big"), (what, i)


@pytest.mark.parametrize("mode", MODE_IDS)
def test_golden_synthetic_vectors(env, golden, oracle, mode):
    vecs = golden["synthetic"]
    stride = max(v["length"] for v in vecs) + 4096
    stride = (stride + 4095) // 4096 * 4096
    host = np.zeros(stride * len(vecs), dtype=np.uint8)
    for i, v in enumerate(vecs):
        host[i * stride:i * stride + v["length"]] = oracle.fill_synthetic(v["length"], v["seed"])
    buf = device_buffer(env, host)
    b = env["DeviceBatch"](buf.data_ptr(), [i * stride for i in range(len(vecs))], [v["length"] for v in vecs],
                           ctx=env["ctx"])
    b.run(_modes(env)[mode])
    assert (b.status_host() == 0).all()
    for v, sha, crc in zip(vecs, b.sha1_hex(), b.crc_sum()):
        assert sha == v["sha1"], v["length"]
        assert "%08x" % crc == v["crc32"], v["length"]


@pytest.mark.parametrize("mode", MODE_IDS)
def test_kat_strings(env, golden, mode):
    vecs = golden["kat"]
    stride = 1024
    host = np.zeros(stride * len(vecs), dtype=np.uint8)
    for i, v in enumerate(vecs):
        b = v["text"].encode()
        host[i * stride:i * stride + len(b)] = np.frombuffer(b, dtype=np.uint8)
    buf = device_buffer(env, host)
    b = env["DeviceBatch"](buf.data_ptr(), [i * stride for i in range(len(vecs))],
                           [len(v["text"].encode()) for v in vecs], ctx=env["ctx"])
    b.run(_modes(env)[mode])
    for v, sha, crc in zip(vecs, b.sha1_hex(), b.crc_sum()):
        assert sha == v["sha1"] and "%08x" % crc == v["crc32"], v["text"]


@pytest.mark.parametrize("mode", MODE_IDS)
def test_misaligned_offsets(env, oracle, mode):
    rng = random.Random(11)
    n = 96
    lengths = [rng.choice([0, 1, 63, 64, 65, 200, 4095, 4096 + 3, 70000, 300001]) for _ in range(n)]
    offsets, pos = [], 0
    for L in lengths:
        pos += rng.randint(0, 17)
        offsets.append(pos)
        pos += L
    host = oracle.fill_synthetic(pos + 64, 321)
    buf = device_buffer(env, host)
    states = env["fresh_states"](n)
    b = env["DeviceBatch"](buf.data_ptr(), offsets, lengths, ctx=env["ctx"])
    b.run(_modes(env)[mode])
    datas = [host[o:o + L].tobytes() for o, L in zip(offsets, lengths)]
    check_batch(b, oracle, datas, states, np.zeros(n, np.uint32), what="misaligned")


def midstream_states(oracle, env, n, rng):
    """States after a random prefix write (nx in 0..63, stale x bytes), plus random CRC states."""
    states = env["fresh_states"](n)
    crcs = np.zeros(n, np.uint32)
    for i in range(n):
        s = oracle.Sha1()
        for _ in range(rng.randint(0, 3)):
            s.write(bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 150))))
        states[i]["h"] = list(s.st.h)
        states[i]["x"] = np.frombuffer(bytes(s.st.x), dtype=np.uint8)
        states[i]["nx"] = s.st.nx
        states[i]["len"] = s.st.len
        crcs[i] = rng.getrandbits(32)
    return states, crcs


@pytest.mark.parametrize("mode", MODE_IDS)
@pytest.mark.parametrize("finalize", [True, False])
def test_midstream_states(env, oracle, mode, finalize):
    rng = random.Random(7 + finalize)
    n = 80
    states, crcs = midstream_states(oracle, env, n, rng)
    lengths = [rng.choice([0, 1, 5, 31, 63, 64, 65, 127, 128, 129, 1000, 4096 * 64 + 9, 131072]) for _ in range(n)]
    stride = 262144 + 4096
    host = oracle.fill_synthetic(stride * n, 99)
    buf = device_buffer(env, host)
    offsets = [i * stride + (i % 5) for i in range(n)]
    b = env["DeviceBatch"](buf.data_ptr(), offsets, lengths, states=states, crcs=crcs, finalize=finalize,
                           ctx=env["ctx"])
    b.run(_modes(env)[mode])
    datas = [host[o:o + L].tobytes() for o, L in zip(offsets, lengths)]
    check_batch(b, oracle, datas, states, crcs, finalize=finalize, what=f"midstream-{mode}")


@pytest.mark.parametrize("mode", MODE_IDS)
def test_go_quirk_states(env, oracle, mode):
    """nx == 64 (full pending block), negative nx, nx > 64 (Go panics), nx inconsistent with len."""
    fresh = env["fresh_states"]
    cases = []  # (state, data)
    s = fresh(1)[0].copy()
    s["x"] = np.frombuffer(b"A" * 64, dtype=np.uint8); s["nx"] = 64; s["len"] = 64
    cases += [(s, b""), (s, b"tail"), (s, b"z" * 200)]
    s2 = fresh(1)[0].copy(); s2["nx"] = -7; s2["len"] = 3
    cases += [(s2, b""), (s2, b"q" * 70), (s2, b"q" * 64)]
    s3 = fresh(1)[0].copy(); s3["nx"] = 65
    cases += [(s3, b""), (s3, b"abc")]
    s4 = fresh(1)[0].copy(); s4["nx"] = 3; s4["len"] = 0; s4["x"][:3] = [1, 2, 3]
    cases += [(s4, b""), (s4, b"x" * 61), (s4, b"x" * 200)]
    s5 = fresh(1)[0].copy(); s5["nx"] = 0; s5["len"] = (1 << 64) - 5  # length wraps
    cases += [(s5, b"wrap-around!")]
    n = len(cases)
    states = fresh(n)
    for i, (st, _) in enumerate(cases):
        states[i] = st
    stride = 256
    host = np.zeros(stride * n, dtype=np.uint8)
    for i, (_, d) in enumerate(cases):
        host[i * stride:i * stride + len(d)] = np.frombuffer(d, dtype=np.uint8)
    buf = device_buffer(env, host)
    b = env["DeviceBatch"](buf.data_ptr(), [i * stride for i in range(n)], [len(d) for _, d in cases],
                           states=states, ctx=env["ctx"])
    b.run(_modes(env)[mode])
    check_batch(b, oracle, [d for _, d in cases], states, np.zeros(n, np.uint32), what=f"quirks-{mode}")


@pytest.mark.parametrize("mode", MODE_IDS)
def test_sha_only_and_crc_only(env, oracle, mode):
    n = 10
    lengths = [0, 1, 64, 100, 5000, 65, 63, 4096, 8191, 12345]
    stride = 16384
    host = oracle.fill_synthetic(stride * n, 5)
    buf = device_buffer(env, host)
    offs = [i * stride for i in range(n)]
    b1 = env["DeviceBatch"](buf.data_ptr(), offs, lengths, crc32=False, ctx=env["ctx"])
    b1.run(_modes(env)[mode])
    b2 = env["DeviceBatch"](buf.data_ptr(), offs, lengths, sha1=False, ctx=env["ctx"])
    b2.run(_modes(env)[mode])
    for i, (o, L) in enumerate(zip(offs, lengths)):
        d = host[o:o + L].tobytes()
        assert b1.sha1_hex()[i] == hashlib.sha1(d).hexdigest()
        assert bytes(b1.sums_host()[i][20:]) == b"\0\0\0\0"
        assert b2.crc_sum()[i] == zlib.crc32(d)
        assert bytes(b2.sums_host()[i][:20]) == b"\0" * 20
        assert bytes(b2.sums_host()[i][20:]) == zlib.crc32(d).to_bytes(4, "big")


def test_wide_uniform_phase_sha_only_and_crc_only(env, oracle):
    """WIDE's uniform loop (every lane of a wave has >= 5 blocks left: no per-lane selects) with one
    of the two hashes only: 192 jobs of 8-24 KiB fill three whole waves, so the uniform phase runs
    for SHA-1 alone and for the position-table CRC alone (efes_kernels.hip wide_bulk)."""
    n = 192
    rng = random.Random(77)
    lengths = [8192 + 64 * rng.randint(0, 256) + rng.randint(0, 63) for _ in range(n)]
    stride = 32768
    host = oracle.fill_synthetic(stride * n, 19)
    buf = device_buffer(env, host)
    offs = [i * stride for i in range(n)]
    wide = _modes(env)["wide"]
    b1 = env["DeviceBatch"](buf.data_ptr(), offs, lengths, crc32=False, ctx=env["ctx"])
    b1.run(wide)
    b2 = env["DeviceBatch"](buf.data_ptr(), offs, lengths, sha1=False, ctx=env["ctx"])
    b2.run(wide)
    for i, (o, L) in enumerate(zip(offs, lengths)):
        d = host[o:o + L].tobytes()
        assert b1.sha1_hex()[i] == hashlib.sha1(d).hexdigest(), (i, L)
        assert b2.crc_sum()[i] == zlib.crc32(d), (i, L)


def test_zero_jobs(env):
    env["ctx"].submit(0, 0)
    env["ctx"].sync()


def test_many_small_jobs_auto(env, oracle):
    rng = np.random.default_rng(2)
    n = 5000
    lengths = rng.integers(0, 3000, n)
    offsets = np.concatenate([[0], np.cumsum(lengths)[:-1]])
    host = oracle.fill_synthetic(int(lengths.sum()) + 8, 1234)
    buf = device_buffer(env, host)
    b = env["DeviceBatch"](buf.data_ptr(), offsets, lengths, ctx=env["ctx"])
    b.run()  # AUTO -> FED4 at this count (efes_auto_mode)
    assert (b.status_host() == 0).all()
    shas, crcs = b.sha1_hex(), b.crc_sum()
    for i in range(0, n, 7):
        d = host[offsets[i]:offsets[i] + lengths[i]].tobytes()
        assert shas[i] == hashlib.sha1(d).hexdigest() and crcs[i] == zlib.crc32(d)


@pytest.mark.parametrize("mode", MODE_IDS)
def test_chunked_resume_equals_one_shot(env, golden, oracle, mode):
    """A 4 MiB+1 object sent as PATCH chunks (write.go:126, filereceiver.go:182-226): state carried on device."""
    v = next(v for v in golden["synthetic"] if v["length"] == (4 << 20) + 1)
    host = oracle.fill_synthetic(v["length"], v["seed"])
    buf = device_buffer(env, host)
    torch = env["torch"]
    cuts = [0, 1, 1000, 1 << 20, (1 << 20) + 63, 3 << 20, v["length"]]
    states = env["fresh_states"](1)
    crc = np.zeros(1, np.uint32)
    for a, c in zip(cuts[:-1], cuts[1:]):
        last = c == v["length"]
        b = env["DeviceBatch"](buf.data_ptr(), [a], [c - a], states=states, crcs=crc, finalize=last, ctx=env["ctx"])
        b.run(_modes(env)[mode])
        states = b.states_host().copy()
        crc = b.crc_sum().copy()
    assert b.sha1_hex()[0] == v["sha1"]
    assert "%08x" % crc[0] == v["crc32"]
    del torch


def test_4mib_batch_against_threaded_oracle(env, oracle):
    n, size = 48, 4 << 20
    torch = env["torch"]
    buf = torch.empty(n * size, dtype=torch.uint8, device="cuda:0")
    env["ctx"].fill_synthetic(buf.data_ptr(), buf.numel(), 0xEFE5, torch.cuda.current_stream().cuda_stream)
    b = env["DeviceBatch"](buf.data_ptr(), [i * size for i in range(n)], [size] * n, ctx=env["ctx"])
    b.run(env["efes"].MODE_DEEP)
    host = buf.cpu().numpy()
    _, sha, crc = oracle.hash_many(host, size, np.full(n, size), 8)
    assert b.sha1_hex() == [bytes(r).hex() for r in sha]
    assert (b.crc_sum() == crc).all()
    b.reset()
    b.run(env["efes"].MODE_WIDE)
    assert b.sha1_hex() == [bytes(r).hex() for r in sha]
    assert (b.crc_sum() == crc).all()


def test_device_fill_matches_host_generator(env, oracle):
    torch = env["torch"]
    for n, seed in [(8, 1), (1000, 2), (4097, 3), (1 << 20, 0xEFE5)]:
        buf = torch.zeros(n + 8, dtype=torch.uint8, device="cuda:0")
        env["ctx"].fill_synthetic(buf.data_ptr(), n, seed, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()  # a null-stream handle selects the context's own non-blocking stream
        got = buf.cpu().numpy()
        assert got[:n].tobytes() == oracle.fill_synthetic(n, seed).tobytes()
        assert not got[n:].any()


# ---------------------------------------------------------------- streaming (Go surface)

def test_streaming_state_vectors(env, golden):
    """MarshalText after every Write equals Go's, stale x bytes included (sha1_efes.go:25-38)."""
    h = env["hashing"]
    for case in golden["sha1_states"]:
        d = h.Sha1Digest(reset=case["reset"])
        for w, text in zip(case["writes"], case["texts"]):
            assert d.write(bytes.fromhex(w)) == len(w) // 2
            assert d.marshal_text().decode() == text, case["name"]
        assert d.sum().hex() == case["sum"], case["name"]


def test_sha1_partial_digest(env):
    """sha1_efes_test.go:8-29 through the GPU-backed digest."""
    h = env["hashing"]
    d = h.Sha1Digest(reset=False)
    d.write(b"hello world")
    hex1 = d.sum().hex()
    text = d.marshal_text()
    d2 = h.Sha1Digest(reset=False)
    d2.unmarshal_text(text)
    assert d2.sum().hex() == hex1 == "73e8730e5086d8ced928b654beeb0e5383f9be01"


def test_crc32_partial_digest(env, golden):
    """crc32_efes_test.go:8-29."""
    h = env["hashing"]
    for case in golden["crc32_states"]:
        c = h.new_crc32_ieee()
        for w, text in zip(case["writes"], case["texts"]):
            c.write(bytes.fromhex(w))
            assert c.marshal_text().decode() == text
        c2 = h.new_crc32_ieee()
        c2.unmarshal_text(c.marshal_text())
        assert c2.sum32() == c.sum32() == case["sum32"]
        assert c2.sum() == case["sum32"].to_bytes(4, "big")


def test_sum_is_non_destructive_and_appends(env):
    h = env["hashing"]
    d = h.new_sha1()
    d.write(b"foo")
    assert d.sum(b"prefix") == b"prefix" + hashlib.sha1(b"foo").digest()
    d.write(b"bar")
    assert d.sum().hex() == "8843d7f92416211de9ebb963ff4ce28125932878"  # TestFileReceiver foo+bar
    assert d.size() == 20 and d.block_size() == 64


def test_reset_keeps_stale_x_like_go(env):
    """sha1.go:36-44: Reset does not clear x, so MarshalText still shows the old tail bytes."""
    h = env["hashing"]
    d = h.new_sha1()
    d.write(b"stale bytes here")
    d.reset()
    text = d.marshal_text().decode()
    assert text[:40] == "67452301efcdab8998badcfe10325476c3d2e1f0"
    assert bytes.fromhex(text[40:40 + 32]) == b"stale bytes here"
    assert text[168:] == "0" * 32
    d.write(b"abc")
    assert d.sum().hex() == hashlib.sha1(b"abc").hexdigest()


def test_streaming_errors(env):
    h = env["hashing"]
    efes = env["efes"]
    d = h.new_sha1()
    with pytest.raises(efes.EfesError) as e:
        d.unmarshal_text(b"00" * 99)
    assert e.value.code == efes.EFES_ERR_INVALID_DIGEST
    good = d.marshal_text()
    d.unmarshal_text(good[:168] + b"%016x" % 65 + b"%016x" % 0)
    with pytest.raises(efes.EfesError) as e:
        d.write(b"x")
    assert e.value.code == efes.EFES_ERR_STATE
    d.unmarshal_text(good[:168] + b"%016x" % 3 + b"%016x" % 0)
    with pytest.raises(efes.EfesError) as e:
        d.sum()
    assert e.value.code == efes.EFES_ERR_STATE
    c = h.new_crc32_ieee()
    with pytest.raises(efes.EfesError):
        c.unmarshal_text(b"xyz")


def test_sha1file_script(env, golden):
    """sha1file_test.go:10-41 with the GPU-backed digest."""
    f = golden["sha1file"]
    sf = env["hashing"].Sha1File(io.BytesIO(f["content"].encode()))
    for (seek, n), want in zip(f["script"], f["reads"]):
        assert sf.seek(seek) == seek
        assert sf.read(n).decode() == want
    assert sf.sum().hex() == f["sha1"] == "5d2781d78fa5a97b7bafa849fe933dfc9dc93eba"


def test_fileinfo_json_roundtrip(env):
    """fileinfo.go: offset + digest JSON persisted between PATCHes, resumed, finalized."""
    h = env["hashing"]
    data = bytes(range(256)) * 40
    fi = h.FileInfo()
    fi.digest.write(data[:5000])
    fi.offset = 5000
    s = fi.dumps()
    fi2 = h.FileInfo.loads(s)
    assert fi2.offset == 5000
    fi2.digest.write(data[5000:])
    assert fi2.digest.sha1.sum().hex() == hashlib.sha1(data).hexdigest()
    assert fi2.digest.crc32.sum32() == zlib.crc32(data)


def test_large_streaming_write_flushes(env):
    h = env["hashing"]
    rng = np.random.default_rng(9)
    data = rng.integers(0, 256, (64 << 20) + 777, dtype=np.uint8).tobytes()
    d = h.new_sha1()
    for i in range(0, len(data), 32 * 1024):  # io.Copy granularity
        d.write(data[i:i + 32 * 1024])
    assert d.sum().hex() == hashlib.sha1(data).hexdigest()


# ---------------------------------------------------------------- host-resident ingest (efes_hash_host)

@pytest.mark.parametrize("segment", [64, 4096, 1 << 20])
def test_host_ingest_matches_oracle(env, oracle, segment):
    """Bytes start in host memory (filereceiver.go:208-209 reads a socket): segmented H2D + hash."""
    from efes_amd.batch import HostBatch
    rng = random.Random(segment)
    lengths = [0, 1, 63, 64, 65, 1000, 4096, 70001, 300000] + [rng.randint(0, 200000) for _ in range(23)]
    offsets, pos = [], 0
    for L in lengths:
        offsets.append(pos)
        pos += L + rng.randint(0, 9)
    host = oracle.fill_synthetic(pos + 8, 77)  # ordinary (pageable) host memory
    hb = HostBatch(host.ctypes.data, offsets, lengths, ctx=env["ctx"])
    st = hb.run(segment)
    assert st.bytes == sum(lengths)
    assert (hb.status[: hb.n] == 0).all()
    for i, (o, L) in enumerate(zip(offsets, lengths)):
        d = host[o:o + L].tobytes()
        assert hb.sha1_hex()[i] == hashlib.sha1(d).hexdigest(), (segment, L)
        assert int(hb.crc_sum()[i]) == zlib.crc32(d), (segment, L)


def test_host_ingest_concurrent_calls_one_context(env, oracle):
    """Four threads in efes_hash_host on one context: they share its copy stream (one hardware
    queue of its own, efes_ingest.cpp) one call at a time, and every digest stays right."""
    import threading
    from efes_amd.batch import HostBatch
    results, errors = {}, []

    def work(t):
        try:
            rng = random.Random(100 + t)
            lengths = [rng.randint(0, 150000) for _ in range(17)] + [64 * (t + 1), 0]
            offsets = np.concatenate([[0], np.cumsum(lengths)[:-1]]).astype(np.uint64).tolist()
            host = oracle.fill_synthetic(sum(lengths) + 8, 900 + t)
            hb = HostBatch(host.ctypes.data, offsets, lengths, ctx=env["ctx"])
            hb.run(16384 * (t + 1))
            results[t] = (host, offsets, lengths, hb.sha1_hex(), hb.crc_sum(), hb.status[: hb.n].copy())
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append(repr(e))

    threads = [threading.Thread(target=work, args=(t,)) for t in range(4)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=100)
    assert not errors, errors
    assert sorted(results) == [0, 1, 2, 3]
    for t, (host, offsets, lengths, sha, crc, status) in results.items():
        assert (status == 0).all()
        for i, (o, L) in enumerate(zip(offsets, lengths)):
            d = host[o:o + L].tobytes()
            assert sha[i] == hashlib.sha1(d).hexdigest(), (t, i, L)
            assert int(crc[i]) == zlib.crc32(d), (t, i, L)


def test_host_ingest_pinned_strided_and_resume(env, oracle):
    """Pinned, constant-stride batch (one 2D copy per segment) resumed from mid-stream states."""
    from efes_amd.batch import HostBatch, PinnedHostBuffer
    rng = random.Random(5)
    n, stride, L = 40, 50000, 49999
    buf = PinnedHostBuffer(n * stride, env["ctx"])
    try:
        buf.array[:] = oracle.fill_synthetic(n * stride, 8)
        states, crcs = midstream_states(oracle, env, n, rng)
        hb = HostBatch(buf.ptr, [i * stride for i in range(n)], [L] * n, fresh=False, states=states, crcs=crcs,
                       ctx=env["ctx"])
        seg = 8192
        hb.run(seg)
        datas = [buf.array[i * stride:i * stride + L].tobytes() for i in range(n)]
        for i, d in enumerate(datas):
            # efes_hash_host == one Write per segment; the stale bytes x[nx:64] depend on the
            # Write boundaries (sha1.go:75-77), so the oracle replays the same boundaries.
            e_status, e_state, e_crc, e_sum = oracle_expect(oracle, states[i], d, int(crcs[i]), writes=seg)
            assert hb.status[i] == e_status
            assert list(hb.states[i]["h"]) == e_state["h"] and int(hb.states[i]["nx"]) == e_state["nx"]
            assert int(hb.states[i]["len"]) == e_state["len"] and bytes(hb.states[i]["x"]) == e_state["x"]
            assert int(hb.crcs[i]) == e_crc
            if e_sum is not None:
                assert bytes(hb.sums[i][:20]) == e_sum
    finally:
        buf.free()


# ---------------------------------------------------------------- concurrent uploads (efes_queue)

def test_upload_queue_concurrent_threads(env, oracle):
    """16 threads, 48 uploads, io.Copy-like Write sizes; sums and MarshalText equal the oracle's
    after the SAME Write calls (stale tail bytes included)."""
    import threading
    from efes_amd.uploads import UploadQueue
    rng = random.Random(21)
    plans = []
    for u in range(48):
        total = rng.choice([0, 1, 63, 64, 65, 1000, 70000, 1 << 20, (3 << 20) + 7, rng.randint(0, 5 << 20)])
        data = oracle.fill_synthetic(total, 1000 + u).tobytes()
        cuts, pos = [], 0
        while pos < total:
            n = min(total - pos, rng.choice([1, 7, 64, 4096, 32 * 1024, 32 * 1024, 200000]))
            cuts.append((pos, n))
            pos += n
        plans.append((data, cuts))
    results = [None] * len(plans)
    errors = []
    with UploadQueue(env["ctx"], chunk_bytes=256 * 1024, max_chunks=64, max_uploads=48) as q:
        def worker(idx):
            try:
                for i in range(idx, len(plans), 16):
                    data, cuts = plans[i]
                    up = q.open()
                    for a, n in cuts:
                        assert up.write(data[a:a + n]) == n
                    mid = up.marshal_text()
                    results[i] = (up.sums(), mid, up.sums())
                    up.close()
            except Exception as e:  # pragma: no cover - reported below
                errors.append(repr(e))
        ths = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
    assert not errors, errors
    for (data, cuts), ((sha, crc), (mt_sha, mt_crc), again) in zip(plans, results):
        assert sha.hex() == hashlib.sha1(data).hexdigest() and crc == zlib.crc32(data)
        assert again == (sha, crc)  # Sum is non-destructive
        o = oracle.Sha1()
        for a, n in cuts:
            o.write(data[a:a + n])
        assert mt_sha.decode() == o.marshal_text()
        assert mt_crc.decode() == "%08x" % zlib.crc32(data)


def test_upload_resume_and_quirks(env, oracle):
    """Open from a saved .info state (fileinfo.go:29-58), continue, and Go's panic states."""
    from efes_amd._lib import Sha1State
    from efes_amd.uploads import UploadQueue
    with UploadQueue(env["ctx"], chunk_bytes=4096, max_chunks=8, max_uploads=4) as q:
        first, rest = b"a" * 1000, bytes(range(256)) * 300
        o = oracle.Sha1()
        o.write(first)
        st = Sha1State()
        st.h[:] = list(o.st.h)
        st.x[:] = bytes(o.st.x)
        st.nx, st.len = o.st.nx, o.st.len
        up = q.open(st, zlib.crc32(first))
        up.write(rest)
        sha, crc = up.sums()
        assert sha.hex() == hashlib.sha1(first + rest).hexdigest() and crc == zlib.crc32(first + rest)
        up.close()
        bad = Sha1State()
        bad.nx = 65
        up = q.open(bad)
        with pytest.raises(env["efes"].EfesError) as e:
            up.write(b"x")
        assert e.value.code == env["efes"].EFES_ERR_STATE
        up.close()
        odd = Sha1State()
        odd.h[:] = list(o.st.h)
        odd.nx, odd.len = 3, 0  # nx inconsistent with len: Go's checkSum panics (sha1.go:107-109)
        up = q.open(odd)
        with pytest.raises(env["efes"].EfesError) as e:
            up.sums()
        assert e.value.code == env["efes"].EFES_ERR_STATE
        up.close()


def test_host_ingest_many_jobs_wide_path(env, oracle):
    """> 1536 jobs per segment: AUTO picks the lane-per-job kernel for the host pipeline too."""
    from efes_amd.batch import HostBatch
    rng = np.random.default_rng(31)
    n = 2500
    lengths = rng.integers(0, 9000, n)
    offsets = np.concatenate([[0], np.cumsum(lengths)[:-1]]).astype(np.uint64)
    host = oracle.fill_synthetic(int(lengths.sum()) + 8, 4321)
    hb = HostBatch(host.ctypes.data, offsets, lengths, ctx=env["ctx"])
    hb.run(4096)
    assert (hb.status[:n] == 0).all()
    for i in range(0, n, 11):
        d = host[int(offsets[i]):int(offsets[i]) + int(lengths[i])].tobytes()
        assert hb.sha1_hex()[i] == hashlib.sha1(d).hexdigest() and int(hb.crc_sum()[i]) == zlib.crc32(d)


def test_deep_mode_more_jobs_than_resident_waves(env, oracle):
    """DEEP with 3000 jobs: more workgroups than fit at once (one per CU by LDS)."""
    rng = np.random.default_rng(8)
    n = 3000
    lengths = rng.integers(0, 20000, n)
    offsets = np.concatenate([[0], np.cumsum(lengths)[:-1]]).astype(np.uint64)
    host = oracle.fill_synthetic(int(lengths.sum()) + 8, 99)
    buf = device_buffer(env, host)
    b = env["DeviceBatch"](buf.data_ptr(), offsets, lengths, fresh=True, ctx=env["ctx"])
    b.run(env["efes"].MODE_DEEP)
    assert (b.status_host() == 0).all()
    shas, crcs = b.sha1_hex(), b.crc_sum()
    for i in range(0, n, 13):
        d = host[int(offsets[i]):int(offsets[i]) + int(lengths[i])].tobytes()
        assert shas[i] == hashlib.sha1(d).hexdigest() and crcs[i] == zlib.crc32(d)


def test_upload_midstream_state_then_continue(env, oracle):
    """.info save in the middle of an upload (filereceiver.go:226), then more PATCH bytes."""
    from efes_amd.uploads import UploadQueue
    data = oracle.fill_synthetic(3 * 100_000 + 17, 55).tobytes()
    with UploadQueue(env["ctx"], chunk_bytes=8192, max_chunks=16, max_uploads=2) as q:
        up = q.open()
        o = oracle.Sha1()
        for a in range(0, 100_000, 32 * 1024):
            piece = data[a:min(a + 32 * 1024, 100_000)]
            up.write(piece)
            o.write(piece)
        st, crc = up.state()
        mt, _ = up.marshal_text()
        assert mt.decode() == o.marshal_text() and crc == zlib.crc32(data[:100_000])
        up.write(data[100_000:])
        sha, crc2 = up.sums()
        assert sha == hashlib.sha1(data).digest() and crc2 == zlib.crc32(data)
        up.close()
        # a second upload resumed from the exported state gives the same result
        up2 = q.open(st, crc)
        up2.write(data[100_000:])
        assert up2.sums() == (sha, crc2)
        up2.close()


def test_upload_reserve_commit_equals_write(env, oracle):
    """Zero-copy staging (efes_upload_reserve / commit, ABI 3): the same Write sequence through
    reserve + fill + commit and through efes_upload_write gives the same state, MarshalText and
    Sums; a reservation larger than the chunk's room hands the chunk over early; commit(0) is
    Go's empty Write (a pending full tail is compressed); a commit beyond the room is refused."""
    from efes_amd._lib import Sha1State
    from efes_amd.uploads import UploadQueue
    efes = env["efes"]
    rng = random.Random(5)
    data = oracle.fill_synthetic(3 << 20, 77).tobytes()
    with UploadQueue(env["ctx"], chunk_bytes=64 * 1024, max_chunks=16, max_uploads=4) as q:
        for trial in range(6):
            a, b = q.open(), q.open()
            o = oracle.Sha1()
            pos = 0
            while pos < len(data) // (trial + 1):
                n = min(rng.choice([0, 1, 63, 64, 65, 4096, 32 * 1024, 40000, 64 * 1024]), len(data) - pos)
                want = rng.choice([1, n or 1, 32 * 1024, 64 * 1024, 1 << 20])
                a.write(data[pos:pos + n])
                view = b.reserve(want)
                assert len(view) >= min(max(want, 1), 64 * 1024)
                if n > len(view):  # reserve what the piece needs, as saveFile does
                    view = b.reserve(n)
                view[:n] = data[pos:pos + n]
                b.commit(n)
                o.write(data[pos:pos + n])
                pos += n
            assert a.marshal_text() == b.marshal_text()
            assert b.marshal_text()[0].decode() == o.marshal_text()
            assert a.sums() == b.sums() == (hashlib.sha1(data[:pos]).digest(), zlib.crc32(data[:pos]))
            a.close()
            b.close()
        # commit(0) on a pending full tail (nx == 64, only reachable through UnmarshalText)
        o = oracle.Sha1()
        o.write(data[:64])
        st = Sha1State()
        st.h[:] = [0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476, 0xC3D2E1F0]
        st.x[:] = data[:64]
        st.nx, st.len = 64, 64
        up = q.open(st)
        up.reserve(1)
        up.commit(0)
        assert up.sums()[0] == hashlib.sha1(data[:64]).digest()
        view = up.reserve(16)
        with pytest.raises(efes.EfesError) as e:
            up.commit(len(view) + 1)
        assert e.value.code == efes.EFES_ERR_ARG
        # a reservation is good for ONE commit: a second one (a stale pointer) is refused, and so is a
        # commit after a write
        view = up.reserve(64)
        view[:8] = b"12345678"
        up.commit(8)
        with pytest.raises(efes.EfesError) as e:
            up.commit(8)
        assert e.value.code == efes.EFES_ERR_ARG
        stale = up.reserve(64)
        up.write(b"x")
        with pytest.raises(efes.EfesError) as e:
            up.commit(1)
        assert e.value.code == efes.EFES_ERR_ARG
        with pytest.raises(ValueError):  # the Python view of an ended reservation is released
            stale[0] = 1
        up.close()


def test_upload_sum_after_queued_chunks(env, oracle):
    """A Sum whose upload still has chunks waiting for a launch rides on the last one's job
    (Write + Sum of a copy, one launch fewer; efes_queue.cpp): the digests, the state left
    behind (MarshalText), a second Sum and later Writes all equal the oracle's.  A Sum that
    fails there (Go's checkSum panic, sha1.go:107-109) leaves the state usable, as Go's does."""
    from efes_amd._lib import Sha1State
    from efes_amd.uploads import UploadQueue
    efes = env["efes"]
    data = oracle.fill_synthetic(300_000, 9).tobytes()
    with UploadQueue(env["ctx"], chunk_bytes=4096, max_chunks=160, max_uploads=8) as q:
        for cut in (0, 64, 4096, 3 * 4096, 3 * 4096 + 5, 100_000, 150 * 1024):
            up = q.open()
            o = oracle.Sha1()
            for a in range(0, cut, 32 * 1024):  # io.Copy's buffers: several full chunks queued
                up.write(data[a:min(a + 32 * 1024, cut)])
            o.write(data[:cut])
            want = (hashlib.sha1(data[:cut]).digest(), zlib.crc32(data[:cut]))
            assert up.sums() == want
            assert up.marshal_text()[0].decode() == o.marshal_text()
            assert up.sums() == want  # non-destructive
            up.write(data[cut:cut + 5000])
            o.write(data[cut:cut + 5000])
            assert up.sums() == (hashlib.sha1(data[:cut + 5000]).digest(), zlib.crc32(data[:cut + 5000]))
            assert up.marshal_text()[0].decode() == o.marshal_text()
            up.close()
        # nx inconsistent with len (only reachable through UnmarshalText): every Sum panics in Go
        o = oracle.Sha1()
        o.st.nx, o.st.len = 3, 0
        st = Sha1State()
        st.h[:] = list(o.st.h)
        st.nx, st.len = 3, 0
        up = q.open(st)
        up.write(data[:8 * 4096])
        o.write(data[:8 * 4096])
        with pytest.raises(efes.EfesError) as e:
            up.sums()
        assert e.value.code == efes.EFES_ERR_STATE
        assert up.marshal_text()[0].decode() == o.marshal_text()
        up.close()


def test_upload_queue_limits(env):
    from efes_amd.uploads import UploadQueue
    efes = env["efes"]
    with pytest.raises(efes.EfesError):
        UploadQueue(env["ctx"], chunk_bytes=4096, max_chunks=4, max_uploads=4)  # needs max_uploads < max_chunks
    with UploadQueue(env["ctx"], chunk_bytes=4096, max_chunks=4, max_uploads=2) as q:
        a, b = q.open(), q.open()
        with pytest.raises(efes.EfesError) as e:
            q.open()
        assert e.value.code == efes.EFES_ERR_NOMEM
        # back-pressure: more bytes than the staging pool holds, from one upload
        blob = bytes(range(256)) * 200
        for _ in range(5):
            a.write(blob)
        assert a.sums()[0] == hashlib.sha1(blob * 5).digest()
        a.close()
        b.close()


def test_bench_emits_driver_json(env):
    """bench.py's contract keys on a tiny configuration (the driver parses this line).

    The child diagnoses its own stall (round 5's r05_check hang lost the child's stack): it runs
    with faulthandler armed (`--watchdog`: every thread's stack to stderr before this test gives
    up), logs each leg's start and end to stderr, and is killed with its whole process group at
    CHILD_S -- before pytest's own 120-s limit -- so the assertion message carries its stderr and
    says whether the JSON line was printed (a stall after it is the process's exit, not a leg)."""
    import json
    import os
    import signal
    import subprocess
    import sys
    # budget: 70.7 s with every leg at its default points on the r06_check box (patch_latency 25.5 s and
    # drain_path 15.6 s of it, CPU-bound harnesses); their shortest points keep each leg exercised
    CHILD_S, WATCHDOG_S = 108, 95
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-X", "faulthandler", os.path.join(root, "bench.py"), "--chunks", "16",
           "--chunk-bytes", "65536", "--steps", "2", "--warmup", "1", "--cpu-seconds", "0.1", "--segment-bytes", "16384",
           "--mixed-leg", "off", "--uploads-leg", "off", "--latency-uploads", "1,16", "--drain-workers", "1,64",
           "--watchdog", str(WATCHDOG_S)]
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, start_new_session=True)
    try:
        out, err = p.communicate(timeout=CHILD_S)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)  # bench.py and the harness binaries it started
        out, err = p.communicate()
        printed = any(line.startswith("{") for line in out.splitlines())
        pytest.fail(f"bench.py did not exit within {CHILD_S} s (JSON line printed: {printed}); its stderr:\n"
                    f"{err[-12000:]}")
    assert p.returncode == 0, f"bench.py exited {p.returncode}; its stderr:\n{err[-12000:]}"
    d = json.loads(out.strip().splitlines()[-1])
    print("leg seconds:", d.get("leg_seconds"))  # the test's time budget, per leg (-s / the log shows it)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["steps"] == 2 and d["n_gpus"] == 1 and d["value"] > 0
    assert d["roofline"]["bound"] == "hbm" and 0 < d["roofline"]["frac"] < 1
    assert d["cpu_baseline"]["digests_match_gpu"] and d["host_inclusive"]["digests_match_device_path"]
    kernels = [p["kernel"] for p in d["concurrency"]["points"]]
    assert kernels[:2] == ["deep_kernel", "fed_kernel<4, 2>"] and kernels[-1] == "wide_kernel"


def test_streaming_digests_batch_across_threads(env, oracle):
    """Unchanged Go-surface digests (MultiWriter(CRC32, Sha1) per request) from 12 threads:
    they share the context's digest queue, so their Writes batch into common launches."""
    import threading
    h = env["hashing"]
    rng = random.Random(3)
    jobs = []
    for i in range(36):
        n = rng.choice([0, 5, 64, 1000, 65536, 300001, rng.randint(0, 2 << 20)])
        jobs.append(oracle.fill_synthetic(n, 500 + i).tobytes())
    res = [None] * len(jobs)
    errs = []

    def worker(t):
        try:
            for i in range(t, len(jobs), 12):
                sha, crc = h.new_sha1(), h.new_crc32_ieee()
                data = jobs[i]
                for a in range(0, len(data), 32 * 1024):  # io.Copy buffers through the MultiWriter
                    crc.write(data[a:a + 32 * 1024])
                    sha.write(data[a:a + 32 * 1024])
                res[i] = (sha.sum().hex(), crc.sum32(), sha.marshal_text().decode())
        except Exception as e:  # pragma: no cover
            errs.append(repr(e))
    ths = [threading.Thread(target=worker, args=(t,)) for t in range(12)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errs, errs
    for data, (sha, crc, mt) in zip(jobs, res):
        assert sha == hashlib.sha1(data).hexdigest() and crc == zlib.crc32(data)
        o = oracle.Sha1()
        for a in range(0, len(data), 32 * 1024):
            o.write(data[a:a + 32 * 1024])
        assert mt == o.marshal_text()


def test_streaming_full_tail_empty_write(env, oracle):
    """nx == 64 then an empty Write: Go compresses the pending block (sha1.go:61-69)."""
    h = env["hashing"]
    o = oracle.Sha1()
    o.st.x[:] = bytes(range(64))
    o.st.nx, o.st.len = 64, 64
    text = o.marshal_text()
    d = h.new_sha1()
    d.unmarshal_text(text.encode())
    d.write(b"")
    o.write(b"")
    assert d.marshal_text().decode() == o.marshal_text()
    assert d.sum().hex() == o.hexdigest()


def test_streaming_sum_keeps_full_tail_pending(env, oracle):
    """Sum right after UnmarshalText of an nx == 64 state works on a copy (sha1.go:82-87): the
    pending block stays pending, so MarshalText is unchanged until the next Write."""
    h = env["hashing"]
    o = oracle.Sha1()
    o.st.x[:] = bytes(range(100, 164))
    o.st.nx, o.st.len = 64, 64
    text = o.marshal_text()
    d = h.new_sha1()
    d.unmarshal_text(text.encode())
    assert d.sum().hex() == o.hexdigest()
    assert d.marshal_text().decode() == o.marshal_text() == text
    d.write(b"more")
    o.write(b"more")
    assert d.marshal_text().decode() == o.marshal_text()
    assert d.sum().hex() == o.hexdigest()


def test_streaming_failed_sum_leaves_digest_usable(env, oracle):
    """A Sum that Go would panic on (checkSum, sha1.go:107-109) runs on a copy: MarshalText and
    later Writes still behave as Go's."""
    h = env["hashing"]
    efes = env["efes"]
    o = oracle.Sha1()
    o.st.x[:3] = b"\x01\x02\x03"
    o.st.nx, o.st.len = 3, 0  # nx inconsistent with len: the padding never lands on a block edge
    text = o.marshal_text()
    d = h.new_sha1()
    d.unmarshal_text(text.encode())
    with pytest.raises(efes.EfesError) as e:
        d.sum()
    assert e.value.code == efes.EFES_ERR_STATE
    assert d.marshal_text().decode() == text
    d.write(b"y" * 200)
    o.write(b"y" * 200)
    assert d.marshal_text().decode() == o.marshal_text()
    with pytest.raises(efes.EfesError):  # len is still inconsistent with nx
        d.sum()
    assert d.marshal_text().decode() == o.marshal_text()


@pytest.mark.parametrize("mode", MODE_IDS)
def test_sum_only_jobs_leave_states(env, oracle, mode):
    """EFES_JOB_SUM_ONLY: the Sum of each in-state, states never written back (sha1.go:82-87)."""
    rng = random.Random(23)
    n = 40
    states, crcs = midstream_states(oracle, env, n, rng)
    states[0]["x"] = np.arange(64, dtype=np.uint8); states[0]["nx"] = 64; states[0]["len"] = 64
    states[1]["nx"] = 5; states[1]["len"] = 0  # Go panics in checkSum
    buf = device_buffer(env, np.zeros(64, np.uint8))
    b = env["DeviceBatch"](buf.data_ptr(), [0] * n, [0] * n, states=states, crcs=crcs, sum_only=True,
                           ctx=env["ctx"])
    b.run(_modes(env)[mode])
    status, st, crc, sums = b.status_host(), b.states_host(), b.crc_sum(), b.sums_host()
    for i in range(n):
        assert bytes(st[i].tobytes()) == bytes(states[i].tobytes()), (mode, i)
        assert int(crc[i]) == int(crcs[i]), (mode, i)
        o = oracle.Sha1(reset=False)
        o.st.h[:] = [int(v) for v in states[i]["h"]]
        o.st.x[:] = bytes(states[i]["x"])
        o.st.nx, o.st.len = int(states[i]["nx"]), int(states[i]["len"])
        src, digest = o.sum()
        if src:
            assert status[i] == env["efes"].EFES_ERR_STATE, (mode, i)
            continue
        assert status[i] == 0, (mode, i)
        assert bytes(sums[i][:20]) == digest, (mode, i)
        assert bytes(sums[i][20:]) == int(crcs[i]).to_bytes(4, "big"), (mode, i)


def test_host_ingest_zero_copy(env, oracle):
    """EFES_HOST_ZERO_COPY: the kernel reads pinned host chunks in place; pageable data is refused."""
    from efes_amd._lib import EFES_HOST_ZERO_COPY
    from efes_amd.batch import HostBatch, PinnedHostBuffer
    rng = random.Random(12)
    lengths = [0, 1, 64, 65, 4095, 100000] + [rng.randint(0, 300000) for _ in range(40)]
    offsets, pos = [], 0
    for L in lengths:
        offsets.append(pos)
        pos += L + rng.randint(0, 7)
    buf = PinnedHostBuffer(pos + 8, env["ctx"])
    try:
        buf.array[:] = oracle.fill_synthetic(pos + 8, 6)
        rngs = random.Random(2)
        states, crcs = midstream_states(oracle, env, len(lengths), rngs)
        hb = HostBatch(buf.ptr, offsets, lengths, fresh=False, states=states, crcs=crcs, ctx=env["ctx"])
        st = hb.run(EFES_HOST_ZERO_COPY)
        assert st.segments == 1 and st.bytes == sum(lengths)
        for i, (o, L) in enumerate(zip(offsets, lengths)):
            d = buf.array[o:o + L].tobytes()
            e_status, e_state, e_crc, e_sum = oracle_expect(oracle, states[i], d, int(crcs[i]))
            assert hb.status[i] == e_status
            assert list(hb.states[i]["h"]) == e_state["h"] and bytes(hb.states[i]["x"]) == e_state["x"]
            assert int(hb.crcs[i]) == e_crc
            if e_sum is not None:
                assert bytes(hb.sums[i][:20]) == e_sum
    finally:
        buf.free()
    pageable = oracle.fill_synthetic(4096, 1)
    hb = HostBatch(pageable.ctypes.data, [0], [4096], ctx=env["ctx"])
    with pytest.raises(env["efes"].EfesError) as e:
        hb.run(EFES_HOST_ZERO_COPY)
    assert e.value.code == env["efes"].EFES_ERR_ARG


@pytest.mark.parametrize("lanes", [4, 8, 16, 32, "fed4", "fed4e"])
def test_group_joint_phase_mixed_lengths_and_states(env, oracle, lanes):
    """Grouped DEEP: jobs of one wave with different lengths, offsets and mid-stream states.

    Lengths are long enough for the joint phase (S > 0) and leave per-job left-over blocks,
    heads (nx != 0) and tails; some waves mix in short jobs that the cost model keeps out of
    the joint phase.  Wave j holds jobs [j*64/lanes, (j+1)*64/lanes)."""
    from efes_amd._lib import MODE_FED4, MODE_FED4E, MODE_GROUP
    fed = {"fed4": MODE_FED4, "fed4e": MODE_FED4E}
    mode = fed.get(lanes) or MODE_GROUP[lanes]
    lanes = 4 if lanes in fed else lanes  # FED4/FED4E: the grouped layout of GROUP4, fed from other SIMDs
    rng = np.random.default_rng(lanes + (mode in fed.values()) + (mode == MODE_FED4E))
    n = 3 * (64 // lanes) + 5  # three full waves and a partial one
    lengths = []
    for i in range(n):
        if i % 7 == 3:
            lengths.append(int(rng.integers(0, 200)))
        else:
            lengths.append(int(rng.integers(40, 120)) * 64 * lanes + int(rng.integers(0, 130)))
    offsets, pos = [], 0
    for L in lengths:
        pos += int(rng.integers(0, 40))
        offsets.append(pos)
        pos += L
    host = oracle.fill_synthetic(pos + 64, 4242 + lanes)
    buf = device_buffer(env, host)
    states, crcs = midstream_states(oracle, env, n, random.Random(lanes))
    b = env["DeviceBatch"](buf.data_ptr(), offsets, lengths, states=states, crcs=crcs, ctx=env["ctx"])
    b.run(mode)
    datas = [host[o:o + L].tobytes() for o, L in zip(offsets, lengths)]
    check_batch(b, oracle, datas, states, crcs, what=f"mode{mode}-lanes{lanes}")


@pytest.mark.parametrize("force", ["4:40x", "8:24", "16:10x,4:30", "32:6,8:20", "64:3x", "0:0", "16:1000",
                                   "64:2x,32:4"])
def test_planned_batch_forced_parts(env, oracle, force):
    """efes_hash_submit_plan: parts on side streams + the caller's stream, concurrently, some
    of them exclusive (CU-reserving LDS) -- every job lands in exactly one launch."""
    from efes_amd.batch import MODE_PLAN
    rng = np.random.default_rng(5)
    n = 150
    lengths = (np.asarray([64 << 10 << int(k) for k in rng.integers(0, 5, n)]) // 16 + rng.integers(0, 100, n))
    offsets = np.concatenate([[0], np.cumsum(lengths)[:-1]]).astype(np.uint64)
    host = oracle.fill_synthetic(int(lengths.sum()) + 8, 77)
    buf = device_buffer(env, host)
    b = env["DeviceBatch"](buf.data_ptr(), offsets, lengths, fresh=True, ctx=env["ctx"])
    b.make_plan(force)
    assert sum(p[0] for p in b.plan.parts()) == n
    b.run(MODE_PLAN)
    assert (b.status_host() == 0).all()
    shas, crcs = b.sha1_hex(), b.crc_sum()
    for i in range(n):
        dat = host[int(offsets[i]):int(offsets[i]) + int(lengths[i])].tobytes()
        assert shas[i] == hashlib.sha1(dat).hexdigest() and crcs[i] == zlib.crc32(dat), (force, i)


@pytest.mark.parametrize("force", ["1:32x,2:48x,4:40x", "2:20x,64:3x,1:16x", "1:40x,2:40x,8:20x,0:60"])
def test_planned_batch_four_parts_fed_on_torch_stream(env, oracle, force):
    """Plans of four parts with FED lanes (FED4 = 1, FED4E = 2) beside grouped / DEEP / WIDE parts,
    submitted on a non-null torch stream (so the caller's stream is neither the context's nor a
    part stream): every part runs on its own part stream, forked from and joined back into the
    caller's stream, and every job matches hashlib/zlib."""
    from efes_amd.batch import MODE_PLAN
    torch = env["torch"]
    rng = np.random.default_rng(11)
    n = 160
    lengths = (np.asarray([32 << 10 << int(k) for k in rng.integers(0, 5, n)]) // 8 + rng.integers(0, 100, n))
    offsets = np.concatenate([[0], np.cumsum(lengths)[:-1]]).astype(np.uint64)
    host = oracle.fill_synthetic(int(lengths.sum()) + 8, 78)
    buf = device_buffer(env, host)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        b = env["DeviceBatch"](buf.data_ptr(), offsets, lengths, fresh=True, ctx=env["ctx"])
        b.make_plan(force)
        assert b.plan.nparts == 4 and sum(p[0] for p in b.plan.parts()) == n
        assert b.stream() != 0 and b.stream() != env["ctx"].stream
        b.submit(MODE_PLAN)
        st = b.status.cpu()  # ordered on s after the plan's join
    torch.cuda.synchronize()
    assert (st.numpy()[:n] == 0).all()
    shas, crcs = b.sha1_hex(), b.crc_sum()
    for i in range(n):
        dat = host[int(offsets[i]):int(offsets[i]) + int(lengths[i])].tobytes()
        assert shas[i] == hashlib.sha1(dat).hexdigest() and crcs[i] == zlib.crc32(dat), (force, i)


def test_planned_batch_random_lengths(env, oracle):
    """The planner's own plan (no forcing) on a heavy-tailed length mix: every digest correct."""
    from efes_amd.batch import MODE_PLAN
    rng = np.random.default_rng(31)
    n = 3000
    lengths = np.minimum(rng.lognormal(10.0, 2.0, n).astype(np.int64), 6 << 20)
    lengths[rng.integers(0, n, 40)] = 0
    offsets = np.concatenate([[0], np.cumsum(lengths + 17)[:-1]]).astype(np.uint64)
    host = oracle.fill_synthetic(int((lengths + 17).sum()) + 64, 2024)
    buf = device_buffer(env, host)
    b = env["DeviceBatch"](buf.data_ptr(), offsets, lengths, fresh=True, ctx=env["ctx"])
    b.make_plan()
    assert sum(p[0] for p in b.plan.parts()) == n
    b.run(MODE_PLAN)
    assert (b.status_host() == 0).all()
    shas, crcs = b.sha1_hex(), b.crc_sum()
    for i in range(n):
        d = host[int(offsets[i]):int(offsets[i]) + int(lengths[i])].tobytes()
        assert shas[i] == hashlib.sha1(d).hexdigest() and crcs[i] == zlib.crc32(d), (i, int(lengths[i]))


def _spot_check(env, buf, offsets, lengths, shas, crcs, picks):
    """hashlib / zlib on chunks copied back from the device (chunks alias a pool: bytes differ)."""
    for i in picks:
        o, n = int(offsets[i]), int(lengths[i])
        d = buf[o:o + n].cpu().numpy().tobytes()
        assert shas[i] == hashlib.sha1(d).hexdigest() and crcs[i] == zlib.crc32(d), (i, n)


def test_full_size_metric_config_all_shapes_agree(env):
    """BASELINE configs[2] at full size (1024 x 4 MiB, device-filled like bench.py): DEEP, GROUP32
    and WIDE (three different kernels, lane layouts and CRC schemes) give identical digests, and a
    sample matches hashlib/zlib.  Size-independent property at the metric's own size."""
    from efes_amd._lib import MODE_GROUP
    torch = env["torch"]
    n, size = 1024, 4 << 20
    buf = torch.empty(n * size, dtype=torch.uint8, device="cuda:0")
    env["ctx"].fill_synthetic(buf.data_ptr(), buf.numel(), 0xEFE5, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    offsets, lengths = np.arange(n, dtype=np.uint64) * size, np.full(n, size, np.uint64)
    b = env["DeviceBatch"](buf.data_ptr(), offsets, lengths, fresh=True, ctx=env["ctx"])
    got = {}
    for name, mode in [("deep", env["efes"].MODE_DEEP), ("group32", MODE_GROUP[32]), ("wide", env["efes"].MODE_WIDE)]:
        b.reset()
        b.run(mode)
        assert (b.status_host() == 0).all(), name
        got[name] = (b.sha1_hex(), b.crc_sum().copy())
    assert got["deep"][0] == got["group32"][0] == got["wide"][0]
    assert (got["deep"][1] == got["group32"][1]).all() and (got["deep"][1] == got["wide"][1]).all()
    assert len(set(got["deep"][0])) == n  # distinct data per chunk
    _spot_check(env, buf, offsets, lengths, got["deep"][0], got["deep"][1], [0, 1, 511, 1022, 1023])


@pytest.mark.parametrize("mode_name", ["deep", "auto"])
def test_full_size_config1_sha1_only(env, mode_name):
    """BASELINE configs[1] at full size: 1024 x 4 MiB, SHA-1 ONLY (jobs without a CRC state, so
    DEEP's producer runs its do_crc == false branch over whole 4 MiB chunks), device-filled like
    bench.py --sha1-only.  Its digests equal the fused run's SHA-1 digests (and hashlib on spot
    chunks), the Sums' CRC bytes stay zero, and no CRC state is written."""
    torch = env["torch"]
    n, size = 1024, 4 << 20
    buf = torch.empty(n * size, dtype=torch.uint8, device="cuda:0")
    env["ctx"].fill_synthetic(buf.data_ptr(), buf.numel(), 0xEFE5, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    offsets, lengths = np.arange(n, dtype=np.uint64) * size, np.full(n, size, np.uint64)
    mode = env["efes"].MODE_DEEP if mode_name == "deep" else env["efes"].MODE_AUTO
    sha_only = env["DeviceBatch"](buf.data_ptr(), offsets, lengths, crc32=False, fresh=True, ctx=env["ctx"])
    sha_only.crcs.fill_(0x5A)  # a CRC state the jobs do not own must stay untouched
    torch.cuda.synchronize()
    sha_only.run(mode)
    assert (sha_only.status_host() == 0).all()
    fused = env["DeviceBatch"](buf.data_ptr(), offsets, lengths, fresh=True, ctx=env["ctx"])
    fused.run(mode)
    assert sha_only.sha1_hex() == fused.sha1_hex()
    assert (sha_only.sums_host()[:, 20:] == 0).all()
    assert (sha_only.crcs.cpu().numpy() == 0x5A).all()
    shas = sha_only.sha1_hex()
    for i in (0, 1, 777, 1023):
        d = buf[i * size:(i + 1) * size].cpu().numpy().tobytes()
        assert shas[i] == hashlib.sha1(d).hexdigest(), i


def test_full_size_mixed_config_plan_equals_wide(env):
    """BASELINE configs[3] at full size and in the bench's own geometry (efes_amd.chunksize.mixed_geometry:
    65 536 chunks of the eleven ChunkSize classes 64K..64M, 752 GiB at seeded offsets of a 200 GiB
    pool filled with seed 0xEFE5, as bench.py's mixed leg): the planner's concurrent parts and an
    all-WIDE run agree on every digest, and at least 64 chunks match hashlib/zlib on their own bytes --
    the first and last chunk of every size class, of every plan part, the chunks on both sides of
    every part boundary, and seeded extras (12 independent checks were too few)."""
    from efes_amd.batch import MODE_PLAN
    from efes_amd.chunksize import MIXED_CLASSES, mixed_geometry
    torch = env["torch"]
    torch.cuda.empty_cache()
    pool = 200 << 30
    buf = torch.empty(pool, dtype=torch.uint8, device="cuda:0")
    env["ctx"].fill_synthetic(buf.data_ptr(), pool, 0xEFE5, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    sizes, offs = mixed_geometry(65536, pool, 7)
    b = env["DeviceBatch"](buf.data_ptr(), offs, sizes, fresh=True, ctx=env["ctx"])
    b.make_plan()
    parts = b.plan.parts()
    assert len(parts) >= 2  # a real multi-part plan
    b.run(MODE_PLAN)
    assert (b.status_host() == 0).all()
    plan_sha, plan_crc = b.sha1_hex(), b.crc_sum().copy()
    b.reset()
    b.run(env["efes"].MODE_WIDE)
    assert (b.status_host() == 0).all()
    assert b.sha1_hex() == plan_sha and (b.crc_sum() == plan_crc).all()
    # the plan runs the jobs longest-first: sizes are already in that order (a stable sort)
    order, _ = env["ctx"].plan(sizes)
    assert (order == np.arange(65536)).all()
    picks = set()
    for c in MIXED_CLASSES:
        idx = np.flatnonzero(sizes == c)
        picks |= {int(idx[0]), int(idx[-1])}
    start = 0
    for jobs, _mode, _x in parts:
        picks |= {start, start + jobs - 1}
        if start:
            picks |= {start - 1, start}
        start += jobs
    rng = np.random.default_rng(0xC3)
    while len(picks) < 72:
        picks.add(int(rng.integers(0, 65536)))
    assert len(picks) >= 64
    _spot_check(env, buf, offs, sizes, plan_sha, plan_crc, sorted(picks))
    del buf, b
    torch.cuda.empty_cache()


@pytest.mark.parametrize("m", [100_000, 196_608])
def test_wide_paced_ragged_launch_every_job(env, m):
    """WIDE with 2 and 3 waves per SIMD (the paced shape launch_wide picks above 65 536 jobs,
    efes_kernels.hip wide_pace) over RAGGED lengths 0..3000 at unaligned offsets: the ragged
    loop, the tail buffer in dynamic LDS and the per-lane finalisation of every job against
    hashlib/zlib (filereceiver.go:208-209 on each chunk)."""
    torch = env["torch"]
    pool = 64 << 20
    buf = torch.empty(pool, dtype=torch.uint8, device="cuda:0")
    env["ctx"].fill_synthetic(buf.data_ptr(), pool, 0x5EED + m, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    rng = np.random.default_rng(m)
    lengths = rng.integers(0, 3001, m).astype(np.uint64)
    lengths[:7] = [0, 1, 55, 56, 63, 64, 3000]
    offs = rng.integers(0, pool - 3001, m).astype(np.uint64)
    b = env["DeviceBatch"](buf.data_ptr(), offs, lengths, fresh=True, ctx=env["ctx"])
    b.run(env["efes"].MODE_WIDE)
    assert (b.status_host() == 0).all()
    shas, crcs = b.sha1_hex(), b.crc_sum()
    host = buf.cpu().numpy()
    for i in range(m):
        d = host[int(offs[i]):int(offs[i]) + int(lengths[i])].tobytes()
        assert shas[i] == hashlib.sha1(d).hexdigest() and crcs[i] == zlib.crc32(d), (i, len(d))


def test_full_size_ingest_launch_wide_equals_group4(env):
    """One BASELINE configs[4] launch at full size (196 608 x 4 MiB, chunks aliasing pool slots as
    bench.py's ingest leg does): WIDE (the shape AUTO picks) and GROUP4 agree on every digest,
    chunks that alias the same slot get the same digest, and a sample matches hashlib/zlib."""
    from efes_amd._lib import MODE_GROUP
    torch = env["torch"]
    chunk, slots, m = 4 << 20, 2048, 196608
    buf = torch.empty(slots * chunk, dtype=torch.uint8, device="cuda:0")
    env["ctx"].fill_synthetic(buf.data_ptr(), buf.numel(), 0xEFE5, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    idx = (np.arange(m, dtype=np.uint64) + np.uint64(7919)) % np.uint64(slots)
    offs, lengths = idx * np.uint64(chunk), np.full(m, chunk, np.uint64)
    b = env["DeviceBatch"](buf.data_ptr(), offs, lengths, fresh=True, ctx=env["ctx"])
    assert env["hashing"].lib().efes_auto_mode(env["ctx"].handle, m) == env["efes"].MODE_WIDE
    b.run(env["efes"].MODE_WIDE)
    assert (b.status_host() == 0).all()
    wide_sha, wide_crc = b.sha1_hex(), b.crc_sum().copy()
    b.reset()
    b.run(MODE_GROUP[4])
    assert (b.status_host() == 0).all()
    assert b.sha1_hex() == wide_sha and (b.crc_sum() == wide_crc).all()
    for i in (0, 1, 2047, 100000):
        assert wide_sha[i] == wide_sha[i + slots] and wide_crc[i] == wide_crc[i + slots]
    assert len(set(wide_sha)) == slots
    _spot_check(env, buf, offs, lengths, wide_sha, wide_crc, [0, 1, 65535, m - 1])


def test_full_size_ingest_segmented_as_benched(env):
    """BASELINE configs[4] exactly as bench.py's ingest leg runs it since round 3 (bench.py ingest
    workload, --ingest-segment 1 MiB): 196 608 chunks of 4 MiB, each arriving as four 1 MiB segment
    Writes from a 192 GiB buffer of distinct bytes (chunk j = its 1 MiB segment, four times), the
    states resident in HBM between the four launches -- the first EFES_JOB_INIT, the last
    EFES_JOB_FINALIZE: the per-PATCH resume of filereceiver.go:182-226 at full occupancy -- in WIDE
    (AUTO's shape at this count, paced at three waves per SIMD), against GROUP4 running the same
    four segments on states of its own: every digest and CRC agrees, and 8 chunks (the first and
    the last job among them) match hashlib/zlib of the 4 MiB they stand for."""
    from efes_amd._lib import MODE_GROUP
    torch = env["torch"]
    seg, m, nseg = 1 << 20, 196608, 4
    buf = torch.empty(m * seg, dtype=torch.uint8, device="cuda:0")
    env["ctx"].fill_synthetic(buf.data_ptr(), buf.numel(), 0x1A6E57, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    offs, lengths = np.arange(m, dtype=np.uint64) * np.uint64(seg), np.full(m, seg, np.uint64)
    assert env["hashing"].lib().efes_auto_mode(env["ctx"].handle, m) == env["efes"].MODE_WIDE
    got = {}
    for mode in (env["efes"].MODE_WIDE, MODE_GROUP[4]):
        base = env["DeviceBatch"](buf.data_ptr(), offs, lengths, fresh=False, ctx=env["ctx"])
        for k in range(nseg):
            base.variant(fresh=k == 0, finalize=k == nseg - 1).run(mode)
        assert (base.status_host() == 0).all(), mode
        got[mode] = (base.sha1_hex(), base.crc_sum().copy())
        del base
    (ws, wc), (gs, gc) = got[env["efes"].MODE_WIDE], got[MODE_GROUP[4]]
    assert ws == gs and (wc == gc).all()
    assert len(set(ws)) == m  # distinct bytes, distinct digests
    for j in (0, 1, 4095, 65535, 65536, 131071, 131072, m - 1):
        chunk = buf[j * seg:(j + 1) * seg].cpu().numpy().tobytes() * nseg
        assert ws[j] == hashlib.sha1(chunk).hexdigest() and int(wc[j]) == zlib.crc32(chunk), j
    del buf
    torch.cuda.empty_cache()


def test_loaded_library_is_built_from_these_sources(env):
    """The libefeshash.so this GPU process loaded was built from the sources in this tree (efes_build_id()
    == efes_amd.build.source_id()): a stale prebuilt library shipped with the tree fails here."""
    from efes_amd import _lib, build
    assert _lib.lib().efes_build_id().decode() == build.source_id()
