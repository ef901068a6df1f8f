"""The unchanged Go surface as bench.py's go_surface_path leg drives it (tools/bench_go_surface: the
calls of INTEGRATION.md §2's hash_gpu.go under filereceiver.go's saveFile -- pooled NewSha1 +
NewCRC32IEEE per PATCH, UnmarshalText of the saved .info, 32 KiB CRC-then-SHA-1 Writes of the same
buffer, MarshalText or Sum), checked here against the CPU oracle and hashlib/zlib:
  * every saved .info text of the resumed PATCHes equals the oracle's after the same Writes;
  * every final Sum equals hashlib/zlib of the object;
  * fused (default): each byte staged and hashed once, every PATCH's pair bound, nothing split;
  * unfused (the SHA-1 digest written from an equal copy of each buffer, so the pair never binds):
    the same texts and digests, each byte hashed twice.
"""
import hashlib
import json
import os
import subprocess
import zlib

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tools", "bench_go_surface")


def _xorshift(n: int) -> bytes:  # the bytes tools/bench_go_surface.cpp hashes
    out = bytearray(n)
    z, m = 0x9E3779B97F4A7C15, (1 << 64) - 1
    for i in range(n):
        z ^= (z << 13) & m
        z ^= z >> 7
        z ^= (z << 17) & m
        out[i] = z & 0xFF
    return bytes(out)


@pytest.mark.parametrize("writes", ["same", "copy"])
def test_go_surface_harness_against_oracle(tmp_path, oracle, writes):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if not os.path.exists(EXE):
        pytest.fail(f"{EXE} not built (__graft_entry__.build())")
    size, write, patches, threads, uploads, k = (1 << 20) + 12345, 32 << 10, 5, 8, 96, 6
    texts = tmp_path / "texts.txt"
    r = subprocess.run([EXE, str(threads), str(uploads), str(size), str(write), str(k), str(patches), "64", "256",
                        str(texts), writes], capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout + r.stderr
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["errors"] == 0 and res["all_equal"], res
    data = _xorshift(size)
    assert res["sum_sha1_crc32"] == hashlib.sha1(data).hexdigest() + "%08x" % zlib.crc32(data)
    # the .info states after PATCHes 1..4, as the oracle computes them after the same 32 KiB Writes
    cut = [size * p // patches for p in range(patches + 1)]
    sha, crc = oracle.Sha1(), oracle.Crc32()
    lines = texts.read_text().split("\n")
    for p in range(patches - 1):
        for a in range(cut[p], cut[p + 1], write):
            piece = data[a:min(a + write, cut[p + 1])]
            crc.write(piece)
            sha.write(piece)
        assert lines[p] == f"{sha.marshal_text()} {crc.marshal_text()}", p
    if writes == "same":
        assert res["hashed_bytes_per_byte"] == 1.0 and res["fused_bytes_per_byte"] == 1.0, res
        assert res["pairs"] == uploads * patches and res["settles"] == 0, res
    else:
        assert res["hashed_bytes_per_byte"] == 2.0 and res["pairs"] == 0, res


@pytest.mark.parametrize("ncontexts", [2, 8])
def test_go_surface_harness_over_a_pool_of_contexts(ncontexts):
    """the Go-surface harness opens its contexts as hash_gpu.go's pool() does --
    every visible GPU by default, here the ordinal list "0,0" or eight times 0 (contexts of GPU 0 stand
    in for the GPUs of one server process, up to an 8-GPU node's pool of eight digest queues) -- and
    reports per-device launches, jobs and bytes.  Every context hashes, their bytes add up to the run's,
    and every Sum equals hashlib/zlib."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if not os.path.exists(EXE):
        pytest.fail(f"{EXE} not built (__graft_entry__.build())")
    size, write, threads, uploads, k = 1 << 20, 32 << 10, 8, 256, 8
    staging = 256 * ncontexts  # 256 MiB per context
    r = subprocess.run([EXE, str(threads), str(uploads), str(size), str(write), str(k), "1", "256", str(staging), "-",
                        "same", ",".join(["0"] * ncontexts)], capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout + r.stderr
    res = json.loads(r.stdout.strip().splitlines()[-1])
    data = _xorshift(size)
    assert res["errors"] == 0 and res["all_equal"], res
    assert res["sum_sha1_crc32"] == hashlib.sha1(data).hexdigest() + "%08x" % zlib.crc32(data)
    assert res["devices_opened"] == ncontexts and res["devices_skipped"] == 0 and res["staging_mib_per_gpu"] == 256, res
    devs = res["devices"]
    assert [d["ordinal"] for d in devs] == [0] * ncontexts and all(d["jobs"] > 0 and d["bytes"] > 0 for d in devs), devs
    assert sum(d["bytes"] for d in devs) == res["hashed_bytes_per_byte"] * uploads * size, devs


def test_uploads_harness_over_queues_of_two_contexts():
    """The uploads harness (bench.py's uploads_path) opens one efes_queue per device that opens and
    places each upload on the queue with the most free slots (go/upload_gpu.go uploadQueue()); with
    the ordinals "0,0" both queues hash, and every Sum equals hashlib/zlib."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    exe = os.path.join(ROOT, "tools", "bench_uploads")
    if not os.path.exists(exe):
        pytest.fail(f"{exe} not built (__graft_entry__.build())")
    size = 1 << 20
    r = subprocess.run([exe, "8", "256", str(size), str(32 << 10), "8", str(256 << 10), "0", "0,0"], capture_output=True,
                       text=True, timeout=110)
    assert r.returncode == 0, r.stdout + r.stderr
    res = json.loads(r.stdout.strip().splitlines()[-1])
    data = _xorshift(size)
    assert res["errors"] == 0 and res["all_sums_equal"], res
    assert res["sum_sha1_crc32"] == hashlib.sha1(data).hexdigest() + "%08x" % zlib.crc32(data)
    devs = res["devices"]
    assert res["devices_opened"] == 2 and [d["ordinal"] for d in devs] == [0, 0], res
    assert all(d["jobs"] > 0 for d in devs) and sum(d["bytes"] for d in devs) == 256 * size, devs
