#!/usr/bin/env python3
"""bench.py -- GiB/s hashed (SHA-1 + CRC-32) on device-resident 4 MiB chunks, 1..N MI355X.

Workload (BASELINE.json configs[2]): per GPU, 1024 independent 4 MiB chunks already resident
in HBM; one step = one fused single-pass SHA-1 + CRC-32 over all of them, each chunk from a
fresh NewSha1()/NewCRC32IEEE() state and finalised on device (the per-chunk digests that
filereceiver.go:208-209 streams every uploaded byte through).  --sha1-only gives configs[1].

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): one process
per GPU, each hashing its own 1024 chunks (weak scaling, per-GPU work queues, no data-path
collective); a barrier + synchronize brackets the timed steps and the time is the max over
ranks (one all_reduce of a scalar, timing only).

Printed on rank 0: ONE JSON line with the driver's keys plus
  roofline     -- the hashing kernel's algorithmic bytes per launch / its average launch time
                  (HIP events on the launch stream), against the 8 TB/s HBM3E peak; traffic
                  from profiles/<round>_traffic.json (rocprofv3 FETCH_SIZE pass) when present;
  cpu_baseline -- the C restatement of the reference (oracle/, kind "port") over the same
                  bytes on the host cores, N=1 rank 0 only, digests checked against the GPU's.
"""
from __future__ import annotations

import argparse
import functools
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

METRIC = "GiB/s hashed (SHA-1+CRC32), device-resident 4 MiB chunks, 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
GiB = 1 << 30


def kernel_names() -> dict:
    """Kernel (rocprof name) of each EFES_MODE_* shape."""
    from efes_amd import MODE_DEEP, MODE_WIDE
    from efes_amd._lib import MODE_FED4, MODE_FED4E, MODE_GROUP

    names = {MODE_DEEP: "deep_kernel", MODE_WIDE: "wide_kernel", MODE_FED4: "fed_kernel<4, 2>",
             MODE_FED4E: "fed_kernel<4, 3>"}
    names.update({v: f"group_kernel<{g}>" for g, v in MODE_GROUP.items()})
    return names


def parse_args(argv=None):
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--chunks", type=int, default=1024, help="chunks per GPU")
    p.add_argument("--chunk-bytes", type=int, default=4 << 20)
    p.add_argument("--mode", choices=["auto", "deep", "wide", "plan", "group4", "group8", "group16", "group32", "fed4",
                                       "fed4e"],
                   default="auto", help="auto: AUTO for chunks4m/ingest, plan (efes_plan_batch) for mixed")
    p.add_argument("--workload", choices=["chunks4m", "mixed", "ingest", "uploads"], default="chunks4m",
                   help="chunks4m = BASELINE configs[1]/[2] (the metric); mixed = configs[3]; ingest = configs[4]")
    p.add_argument("--pool-gib", type=int, default=64, help="device pool aliased by mixed/ingest chunks")
    p.add_argument("--mixed-chunks", type=int, default=65536)
    p.add_argument("--mixed-launches", type=int, default=1,
                   help="deal the longest-first mixed job list round-robin into this many launches")
    p.add_argument("--upload-threads", type=int, default=16)
    p.add_argument("--uploads", type=int, default=1024)
    p.add_argument("--upload-bytes", type=int, default=4 << 20)
    p.add_argument("--write-bytes", type=int, default=32 << 10, help="io.Copy buffer size (32 KiB)")
    p.add_argument("--open-per-thread", type=int, default=64, help="uploads in flight per request thread")
    p.add_argument("--progress", action="store_true",
                   help="synchronize after every step and print progress to stderr (long workloads)")
    p.add_argument("--ingest-tib", type=float, default=10.0)
    p.add_argument("--ingest-scale", type=float, default=1.0)
    p.add_argument("--ingest-batch", type=int, default=196608,
                   help="chunks per launch: 3 WIDE waves per SIMD (132 VGPRs -> 3 resident) x 1024 SIMDs x 64")
    p.add_argument("--ingest-segment", type=int, default=1 << 20,
                   help="ingest: each 4 MiB chunk as Writes of this many bytes, distinct data in every launch "
                        "(0: whole chunks aliasing a --pool-gib pool, the round-1/2 leg)")
    p.add_argument("--sha1-only", action="store_true", help="BASELINE configs[1] (no CRC-32)")
    p.add_argument("--cpu-threads", type=int, default=0, help="cpu_baseline threads (0 = host share, max 16)")
    p.add_argument("--cpu-max-chunks", type=int, default=1024)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--host-inclusive", choices=["auto", "on", "off"], default="auto",
                   help="also time the host-resident path (pinned H2D + hash); auto = N=1 only")
    p.add_argument("--segment-bytes", type=int, default=256 << 10, help="host-inclusive pipeline segment")
    p.add_argument("--ingest-leg", choices=["auto", "on", "off"], default="auto",
                   help="also report BASELINE configs[4]: each GPU's share of 10 TiB, aggregated over all ranks "
                        "(auto = on at every N)")
    p.add_argument("--sha1-leg", choices=["auto", "on", "off"], default="auto",
                   help="also report BASELINE configs[1] (the same chunks, SHA-1 only); auto = N=1 only")
    p.add_argument("--uploads-leg", choices=["auto", "on", "off"], default="auto",
                   help="also report the server path (tools/bench_uploads: 32 request threads x 256 uploads in "
                        "flight, 8192 x 4 MiB, 32 KiB pageable Writes, Sum each); auto = N=1 only")
    p.add_argument("--go-surface-leg", choices=["auto", "on", "off"], default="auto",
                   help="also report the UNCHANGED Go surface (tools/bench_go_surface: hash_gpu.go's calls under "
                        "saveFile, fused MultiWriter pairs, and the SHA-1 Writes from a copy: never fused) at "
                        "uploads_path's concurrency "
                        "(auto: N=1)")
    p.add_argument("--latency-leg", choices=["auto", "on", "off"], default="auto",
                   help="also report per-PATCH latency at 1/16/256 uploads in flight, GPU vs the CPU port (auto: N=1)")
    p.add_argument("--receiver-leg", choices=["auto", "on", "off"], default="auto",
                   help="also report the receiver with files (tools/bench_receiver: saveFile through ServeHTTP, "
                        "768 request threads x 4 MiB PATCHes on tmpfs) and Sha1File read-back (256 threads); auto = N=1 only")
    p.add_argument("--drain-leg", choices=["auto", "on", "off"], default="auto",
                   help="also report the drainer's read-back (sendFile/Sha1File mirror, K files in flight) against "
                        "the CPU port; auto = N=1 only")
    p.add_argument("--concurrency-leg", choices=["auto", "on", "off"], default="auto",
                   help="also report 4 MiB chunks at 1K..192K in flight, one AUTO launch each (auto = N=1 only)")
    p.add_argument("--mixed-leg", choices=["auto", "on", "off"], default="auto",
                   help="also report BASELINE configs[3] (planned mixed-size batch); auto = N=1 only")
    p.add_argument("--span-leg", choices=["auto", "on", "off"], default="auto",
                   help="CRC-32 of one 16 GiB object (efes_crc32_span, SURVEY.md §8(f) row 4); auto = N=1 only")
    p.add_argument("--dist-backend", default="nccl", help="N>1 timing barrier/max only (no data-path collective)")
    p.add_argument("--all-ranks-on-device0", action="store_true",
                   help="rehearse the N>1 path on a 1-GPU box (use with --dist-backend gloo)")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="minimum CPU work in the cpu_baseline sample")
    p.add_argument("--latency-uploads", default="1,16,64,128,192,256",
                   help="patch_latency leg: uploads in flight of each point")
    p.add_argument("--drain-workers", default="1,16,64,128,192,256,512", help="drain_path leg: workers of each point")
    p.add_argument("--watchdog", type=float, default=0.0,
                   help="dump every thread's Python stack to stderr after this many seconds (faulthandler; "
                        "0 = off; the GPU test of this file arms it)")
    return p.parse_args(argv)


class Legs:
    """Runs the side legs one after the other, logging each start and end to stderr (so a stalled
    run names its leg) and keeping their wall seconds for the output line (`leg_seconds`)."""

    def __init__(self):
        self.seconds = {}
        self.t0 = time.perf_counter()

    def run(self, name: str, fn, *a, **kw):
        t = time.perf_counter()
        print(f"[bench] {name}: start at {t - self.t0:.1f} s", file=sys.stderr, flush=True)
        r = fn(*a, **kw)
        self.seconds[name] = round(time.perf_counter() - t, 2)
        print(f"[bench] {name}: done in {self.seconds[name]} s", file=sys.stderr, flush=True)
        return r


def _ints(csv: str) -> tuple:
    return tuple(int(x) for x in csv.split(",") if x.strip())


def host_threads() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        n = os.cpu_count() or 1
    return max(1, min(16, n))  # the GPU box grants 16 host cores per GPU


def load_traffic(kernel: str, workload_key: str):
    """Per-launch HBM bytes of `kernel` measured by rocprofv3 --pmc (tools/pmc_traffic.py)."""
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json"))):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if d.get("kernel") == kernel and d.get("workload_key") == workload_key:
            best = d
    return None if best is None else float(best["bytes_per_launch"])


def config0_cpu(data, chunk: int):
    """BASELINE configs[0]: sha1file.go over one 4 MiB chunk on the CPU path (the oracle's
    Sha1File, 32 KiB reads as io.Copy issues them, one seek-back-and-reread like a retried
    PATCH, sha1file.go:23-49), single thread; the digest is checked against the GPU's."""
    import hashlib

    from oracle import oracle

    host = data[:chunk].cpu().numpy().tobytes()
    best = None
    for _ in range(3):
        f = oracle.Sha1File(host)  # wraps the chunk (the ReadSeeker), outside the timed region
        t0 = time.perf_counter()
        for a in range(0, chunk // 2, 32 << 10):
            f.read(32 << 10)
        f.seek(chunk // 4)  # retry: seek back, bytes up to `calculated` are not hashed again
        while f.read(32 << 10):
            pass
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
        digest = f.sum()
    return {"value": round(chunk / best / (1 << 20), 1), "unit": "MiB/s", "cores": 1, "kind": "port",
            "sample": f"Sha1File over one {chunk >> 20} MiB chunk, 32 KiB reads, one seek-back, best of 3",
            "digest_matches": digest == hashlib.sha1(host).digest()}


def cpu_baseline(batch, data, n_chunks: int, chunk: int, threads: int, do_crc: bool, min_seconds: float = 10.0):
    """The oracle (C restatement of sha1.go block + crc32.go slicingUpdate) over the same chunks."""
    import numpy as np

    from oracle import oracle

    oracle.build()
    m = max(1, min(n_chunks, threads * max(1, n_chunks // threads)))
    host = data[: m * chunk].cpu().numpy()
    lens = np.full(m, chunk, dtype=np.uint64)
    secs, reps = 0.0, 0
    while secs < min_seconds or reps == 0:  # a bounded sample of >= min_seconds of CPU work
        dt, sha, crc = oracle.hash_many(host, chunk, lens, threads)
        secs += dt
        reps += 1
    got = batch.sha1_hex()[:m]
    ok = got == [bytes(r).hex() for r in sha]
    if do_crc:
        ok = ok and bool((batch.crc_sum()[:m] == crc).all())
    return {
        "value": round(reps * m * chunk / secs / GiB, 3),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{reps} pass(es) over {m} x {chunk >> 20} MiB chunks of the same workload (fused SHA-1+CRC32 in"
                  f" filereceiver.go:208 MultiWriter order), one chunk per thread at a time, {secs:.1f} s",
        "digests_match_gpu": bool(ok),
    }


def host_inclusive(ctx, data, n: int, chunk: int, do_crc: bool, segment: int, batch):
    """The same chunks starting in pinned host memory: H2D copies overlapped with hashing (DESIGN_NOTES.md)."""
    from efes_amd._lib import EFES_HOST_ZERO_COPY
    from efes_amd.batch import HostBatch, PinnedHostBuffer

    buf = PinnedHostBuffer(n * chunk, ctx)
    try:
        ctx.copy_to_host(buf.ptr, data.data_ptr(), n * chunk)
        hb = HostBatch(buf.ptr, [i * chunk for i in range(n)], [chunk] * n, crc32=do_crc, ctx=ctx)
        hb.run(segment)  # warm-up (first-touch of the pipeline buffers)
        hb = HostBatch(buf.ptr, [i * chunk for i in range(n)], [chunk] * n, crc32=do_crc, ctx=ctx)
        st = hb.run(segment)
        ok = hb.sha1_hex() == batch.sha1_hex() and (not do_crc or bool((hb.crc_sum() == batch.crc_sum()).all()))
        zc = HostBatch(buf.ptr, [i * chunk for i in range(n)], [chunk] * n, crc32=do_crc, ctx=ctx)
        sz = zc.run(EFES_HOST_ZERO_COPY)
        ok = ok and zc.sha1_hex() == batch.sha1_hex()
    finally:
        buf.free()
    return {"value": round(st.bytes / st.seconds / GiB, 3), "unit": "GiB/s", "segment_bytes": segment,
            "segments": st.segments, "zero_copy_value": round(sz.bytes / sz.seconds / GiB, 3),
            "digests_match_device_path": bool(ok),
            "note": "pinned host chunks: value = hipMemcpyAsync H2D segments (copy stream) overlapped with hashing; "
                    "zero_copy_value = one DEEP launch reading the pinned chunks over PCIe in place; not `value`"}


@functools.lru_cache(maxsize=2)
def _xorshift_bytes(n: int) -> bytes:
    """The byte stream tools/bench_uploads.cpp hashes (xorshift64, low byte of each step)."""
    out = bytearray(n)
    z = 0x9E3779B97F4A7C15
    m = (1 << 64) - 1
    for i in range(n):
        z ^= (z << 13) & m
        z ^= z >> 7
        z ^= (z << 17) & m
        out[i] = z & 0xFF
    return bytes(out)


def uploads_workload(args, ctx):
    """Concurrent uploads through the batching dispatcher (efes_queue), driven natively by
    tools/bench_uploads (built by __graft_entry__.build): --upload-threads request threads each
    run uploads of --upload-bytes as Write calls of --write-bytes (io.Copy's 32 KiB,
    filereceiver.go:209) from pageable memory, then Sum -- the server path end to end (host
    staging, H2D, hashing, per-upload sync point).  Returns the result dict (not the metric)."""
    import hashlib
    import subprocess
    import zlib

    exe = os.path.join(ROOT, "tools", "bench_uploads")
    cmd = [exe, str(args.upload_threads), str(args.uploads), str(args.upload_bytes), str(args.write_bytes),
           str(args.open_per_thread)]
    res = json.loads(subprocess.run(cmd, check=True, capture_output=True, text=True).stdout.strip().splitlines()[-1])
    src = _xorshift_bytes(args.upload_bytes)
    want = hashlib.sha1(src).hexdigest() + "%08x" % zlib.crc32(src)
    res["digests_match"] = res.pop("sum_sha1_crc32") == want and res.pop("all_sums_equal")
    res["note"] = "native request threads: pageable Writes -> pinned staging -> batched launches -> per-upload Sum"
    return res


def go_surface_leg(uploads=None):
    """The drop-in boundary as unchanged Go code calls it (efes_hash.h layer 2; INTEGRATION.md §2's
    hash_gpu.go under filereceiver.go's saveFile), driven natively by tools/bench_go_surface at
    uploads_path's concurrency (32 request threads x 256 uploads in flight, 8 192 x 4 MiB, 32 KiB
    io.Copy buffers): per PATCH efes_sha1_new_pool + efes_crc32_new_pool, efes_crc32_write then
    efes_sha1_write of the SAME buffer (MultiWriter(f, CRC32, Sha1), filereceiver.go:208-209), Sum of
    both.  The library fuses each pair into one upload (efes_stream.cpp); the same run with the SHA-1
    digest written from an equal copy of each buffer (the pair never binds: two uploads, each byte
    staged and hashed twice, round 3's behaviour) is reported beside it.
    Digests checked against hashlib/zlib.  Returns the result dict (not the metric)."""
    import hashlib
    import subprocess
    import zlib

    exe = os.path.join(ROOT, "tools", "bench_go_surface")
    cmd = [exe, "32", "8192", str(4 << 20), str(32 << 10), "256", "1", "256", "8208"]

    def run(writes):
        r = subprocess.run(cmd + ["-", writes], check=True, capture_output=True, text=True, timeout=300)
        return json.loads(r.stdout.strip().splitlines()[-1])

    src = _xorshift_bytes(4 << 20)
    want = hashlib.sha1(src).hexdigest() + "%08x" % zlib.crc32(src)
    res = run("same")
    res["digests_match"] = res.pop("sum_sha1_crc32") == want and res.pop("all_equal")
    un = run("copy")
    res["unfused"] = {"value": un["value"], "unit": "GiB/s", "hashed_bytes_per_byte": un["hashed_bytes_per_byte"],
                      "launches": un["launches"], "digests_match": un["sum_sha1_crc32"] == want and un["all_equal"],
                      "note": "SHA-1 Writes from an equal copy of each buffer: the CRC and SHA-1 digests as two "
                              "uploads"}
    if uploads and uploads.get("value"):
        res["vs_uploads_path"] = round(res["value"] / uploads["value"], 4)
    res["note"] = ("unchanged Go call sequence (hash_gpu.go): pooled NewSha1 + NewCRC32IEEE per PATCH, 32 KiB "
                   "CRC-then-SHA-1 Writes of one buffer, Sum; the pair fused into one upload by the library")
    return res


def patch_latency_leg(uploads=(1, 16, 64, 128, 192, 256)):
    """Per-PATCH latency of one 4 MiB PATCH (saveFile's hashing: MultiWriter CRC-then-SHA-1 Writes in
    32 KiB buffers, then both Sums) with 1, 16 and 256 uploads in flight: the unchanged Go surface on
    the GPU (tools/bench_go_surface, one PATCH per request thread, fused pairs) against the CPU port
    of the same hashing on the box's CPU quota (oracle/patch_cpu, the reference's algorithm; a
    reported baseline).  Both hash the same bytes; digests checked against hashlib/zlib."""
    import hashlib
    import subprocess
    import zlib

    src = _xorshift_bytes(4 << 20)
    want = hashlib.sha1(src).hexdigest() + "%08x" % zlib.crc32(src)

    def run(argv):
        r = subprocess.run(argv, check=True, capture_output=True, text=True, timeout=300)
        return json.loads(r.stdout.strip().splitlines()[-1])

    points = []
    for k in uploads:
        rounds = 20 if k == 1 else 8 if k <= 16 else 6 if k <= 64 else 4
        g = run([os.path.join(ROOT, "tools", "bench_go_surface"), str(k), str(k * rounds), str(4 << 20), str(32 << 10),
                 "1", "1", "256", "1024"])
        c = run([os.path.join(ROOT, "oracle", "patch_cpu"), str(k), str(4 << 20), "3"])
        points.append({"uploads_in_flight": k, "gpu_patch_ms": g["patch_group_ms"], "gpu_GiB/s": g["value"],
                       "cpu_patch_ms": c["patch_ms"], "cpu_GiB/s": c["value"], "cpu_threads_pinned": c["pinned_cpus"],
                       "digests_match": g["sum_sha1_crc32"] == want and g["all_equal"] and
                       c["sum_sha1_crc32"] == want and c["all_equal"]})
    over = next((p["uploads_in_flight"] for p in points if p["gpu_GiB/s"] > p["cpu_GiB/s"]), None)
    cores = points[0]["cpu_threads_pinned"]
    return {"patch_bytes": 4 << 20, "points": points, "gpu_overtakes_cpu_at_uploads": over, "cpu_cores": cores,
            "note": "GPU: unchanged Go surface, one PATCH per request thread; CPU: oracle port of the same hashing "
                    "(kind port) on the quota's cores; latency = one PATCH's Writes + Sums; the efesgpu server "
                    "hashes faster than the pure-Go build from gpu_overtakes_cpu_at_uploads in flight on "
                    "cpu_cores host cores (INTEGRATION.md §1); not `value`"}


def receiver_leg():
    """The Go callers above the ABI, restated in C++ (efes_amd/host/efes_receiver.hpp), driven by
    tools/bench_receiver: request threads run saveFile through FileReceiver::ServeHTTP (file write,
    fsync, the fused upload, .info between PATCHes, digest headers at the end; one PATCH at a time
    per thread, as net/http runs a handler), files on tmpfs when there is one; and Sha1File over a
    file (write.go:69).  Digests checked against hashlib/zlib.  Returns the result dict."""
    import hashlib
    import subprocess
    import tempfile
    import zlib

    import statistics

    exe = os.path.join(ROOT, "tools", "bench_receiver")
    base = "/dev/shm" if os.access("/dev/shm", os.W_OK) else tempfile.gettempdir()
    out = {}

    def run(argv, env=None):
        r = subprocess.run([exe] + argv, check=True, capture_output=True, text=True, timeout=300,
                           env=dict(os.environ, **(env or {})))
        return json.loads(r.stdout.strip().splitlines()[-1])

    src = _xorshift_bytes(4 << 20)
    with tempfile.TemporaryDirectory(dir=base, prefix="efes_receiver_") as d:
        # 768 request threads: the GPU box counts threads against a 1024-process limit, and 1024 of
        # them beside this process's own runtime threads crossed it once (under rocprof); 768
        # leaves ~200 for the runtimes (12.0-19.0 GiB/s at 1024 threads, 12.7-13.1 at 512).
        # Receiver and copy ceiling alternate, three times: the fraction is the median of the pairs.
        recv, copy, copy_res, fracs, ok = [], [], [], [], True
        want = hashlib.sha1(src).hexdigest() + "%08x" % zlib.crc32(src)
        for _ in range(3):
            r = run(["receiver", d, "768", "4", str(4 << 20), str(4 << 20)])
            ok = ok and r.pop("sum_sha1_crc32") == want and r.pop("all_sums_equal")
            c = run(["copy", d, "768", "4", str(4 << 20)])
            recv.append(r)
            copy_res.append(c)
            copy.append(c["value"])
            fracs.append(r["value"] / c["value"])
        res = dict(recv[0])
        res.update({"value": round(statistics.median(x["value"] for x in recv), 3),
                    "values": [x["value"] for x in recv], "copy_ceiling": round(statistics.median(copy), 3),
                    "copy_values": copy, "frac_of_copy": round(statistics.median(fracs), 3),
                    "frac_of_copy_each": [round(f, 3) for f in fracs], "digests_match": bool(ok),
                    "cpu_s_per_gib": [x.get("cpu_s_per_gib") for x in recv],
                    "copy_cpu_s_per_gib": [c.get("cpu_s_per_gib") for c in copy_res]})
        # one more receiver run with saveFile's host-time accounting by phase (efes_receiver.cpp)
        ph = run(["receiver", d, "768", "4", str(4 << 20), str(4 << 20)], {"EFES_RECEIVER_PHASES": "1"})
        res["phases"] = {"value": ph["value"], "cpu_s_per_gib": ph.get("cpu_s_per_gib"),
                         "request_threads_cpu_s_per_gib": ph.get("request_threads_cpu_s_per_gib"),
                         "phase_cpu_s_per_gib": ph.get("phase_cpu_s_per_gib")}
        # the reference's saveFile with its digests on the CPU port (oracle/receiver_cpu: the same
        # file work, SHA-1 + CRC-32 in MultiWriter order on 16 threads = the box's host cores)
        from oracle import oracle

        oracle.build()
        rc = subprocess.run([os.path.join(ROOT, "oracle", "receiver_cpu"), d, "16", "64", str(4 << 20)], check=True,
                            capture_output=True, text=True, timeout=300)
        cres = json.loads(rc.stdout.strip().splitlines()[-1])
        res["cpu_port"] = {"value": cres["value"], "unit": "GiB/s", "cores": 16, "kind": "port",
                           "digests_match": cres["sum_sha1_crc32"] == want and cres["all_sums_equal"],
                           "sample": f"oracle/receiver_cpu: {cres['uploads']} one-PATCH uploads x 4 MiB, saveFile's file "
                                     f"work + SHA-1/CRC-32 on the CPU port, 16 threads, {cres['seconds']} s"}
        res["vs_cpu_port"] = round(res["value"] / cres["value"], 2)
        out["receiver"] = res
        r = run(["sha1file", d, "256", "4", str(4 << 20)])
        r["digests_match"] = r.pop("sum_sha1") == hashlib.sha1(src).hexdigest() and r.pop("all_sums_equal")
        out["sha1file"] = r
    out["note"] = ("receiver: saveFile with the digests on the GPU (median of 3); copy_ceiling: the same PATCHes "
                   "without the digests -- createFile with its .info, io.Copy in 32 KiB reads, fsync, close, "
                   "DeleteFileInfo -- on the same host cores; not `value`")
    return out


def drain_leg(workers=(1, 16, 64, 128, 192, 256, 512), file_bytes: int = 4 << 20, cpu_threads: int = 16,
              files_per_worker: int = 16):
    """The drainer's read-back (drain.go:87-125 -> write.go:68-117 sendFile ->
    sha1file.go): files on tmpfs moved by K concurrent workers through the C++ sendFile/Sha1File
    mirror, every read hashed on the GPU (their streams batched by the digest queue), to a sink
    server; against the CPU port -- the oracle's sha1digest over the same files in 32 KiB reads on
    `cpu_threads` host threads.  Reports the K at which the GPU path overtakes the CPU.  Each worker
    moves `files_per_worker` files one after the other (16: the steady state; with 4 the workers'
    start and the last files' chains -- 46 ms each -- were a third of the run,
    profiles/r03_drain/drain_stats.log)."""
    import hashlib
    import subprocess
    import tempfile

    from oracle import oracle

    exe = os.path.join(ROOT, "tools", "bench_receiver")
    base = "/dev/shm" if os.access("/dev/shm", os.W_OK) else tempfile.gettempdir()
    src = _xorshift_bytes(file_bytes)
    want = hashlib.sha1(src).hexdigest()
    nfiles = 256
    points = []
    with tempfile.TemporaryDirectory(dir=base, prefix="efes_drain_") as d:
        for i in range(nfiles):
            with open(os.path.join(d, f"{i}.fid"), "wb") as f:
                f.write(src)
        for k in workers:
            fids = max(8, files_per_worker * k)
            r = subprocess.run([exe, "drain", d, str(k), str(fids), str(file_bytes), str(nfiles)], check=True,
                               capture_output=True, text=True, timeout=300)
            res = json.loads(r.stdout.strip().splitlines()[-1])
            points.append({"workers": k, "fids": fids, "GiB/s": res["value"],
                           "cpu_s_per_gib": res.get("cpu_s_per_gib"), "jobs_per_launch": res.get("jobs_per_launch"),
                           "digests_match": res["sum_sha1"] == want and res["all_sums_equal"] and not res["errors"]})

        # the CPU port: oracle/drain_cpu (sha1digest's generic block restated in C, 32 KiB reads through
        # Sha1File's Write) on `cpu_threads` pthreads, one file in flight each, over the same files
        oracle.build()
        exe_cpu = os.path.join(ROOT, "oracle", "drain_cpu")
        fids_cpu = 4096
        r = subprocess.run([exe_cpu, d, str(cpu_threads), str(fids_cpu), str(file_bytes), str(nfiles)], check=True,
                           capture_output=True, text=True, timeout=300)
        cres = json.loads(r.stdout.strip().splitlines()[-1])
        cpu = cres["value"]
        ok_cpu = cres["sum_sha1"] == want and cres["all_sums_equal"] and not cres["errors"]
        n_cpu = fids_cpu
    over = next((p["workers"] for p in points if p["GiB/s"] > cpu), None)
    return {"unit": "GiB/s", "file_bytes": file_bytes, "points": points,
            "cpu_port": {"value": round(cpu, 3), "cores": cpu_threads, "kind": "port", "digests_match": bool(ok_cpu),
                         "sample": f"{n_cpu} x {file_bytes >> 20} MiB files (oracle/drain_cpu: sha1digest in 32 KiB "
                                   f"reads, one file per thread at a time, {cres['seconds']} s)"},
            "gpu_overtakes_cpu_at_workers": over,
            "note": "sendFile(Sha1File) per file to a sink server (its SHA-1 answer known), K files in flight; "
                    "one stream is one SHA-1 chain (~90 MB/s), so the GPU needs many files in flight; not `value`"}


def make_workload(args, rank: int, world: int, ctx, device: str, stream):
    """Device-resident inputs + the job batches of one workload.

    chunks4m (default, BASELINE configs[2] / configs[1] with --sha1-only): n x 4 MiB chunks
        packed in HBM, one batch, one launch per step.
    mixed (configs[3]): --mixed-chunks chunks whose sizes are the eleven ChunkSize values
        64K..64M (chunksize.go) drawn uniformly (log-uniform in bytes, seed 7 + rank); they
        alias a --pool-gib device pool at seeded 256-B aligned offsets; jobs are submitted
        longest first so each wave's 64 lanes carry equal lengths. One step = all chunks.
    ingest (configs[4]): this GPU's share of --ingest-tib TiB of 4 MiB chunks on an 8-GPU node
        (fixed per GPU: weak scaling), scaled by --ingest-scale, in launches of
        --ingest-batch chunks aliasing the pool. One step = one launch.
    Returns (data tensor, [DeviceBatch...], bytes per step list, config dict).
    """
    import numpy as np
    import torch

    from efes_amd.batch import DeviceBatch
    from efes_amd.chunksize import mixed_geometry

    kw = dict(sha1=True, crc32=not args.sha1_only, finalize=True, fresh=True, ctx=ctx, device=device)
    seed = 0xEFE5 ^ (rank << 32)
    if args.workload == "chunks4m":
        n, chunk = args.chunks, args.chunk_bytes
        data = torch.empty(n * chunk, dtype=torch.uint8, device=device)
        ctx.fill_synthetic(data.data_ptr(), n * chunk, seed, stream.cuda_stream)
        b = DeviceBatch(data.data_ptr(), np.arange(n, dtype=np.uint64) * chunk, np.full(n, chunk), **kw)
        name = (("1024 x 4 MiB chunks, SHA-1 only (BASELINE configs[1])" if args.sha1_only else
                 "1024 x 4 MiB chunks, fused single-pass SHA-1 + CRC32 (BASELINE configs[2])")
                if (n, chunk) == (1024, 4 << 20) else f"{n} x {chunk} B chunks")
        return data, [b], [n * chunk], {"workload": name, "chunks_per_gpu": n, "chunk_bytes": chunk}
    pool = args.pool_gib << 30
    if args.workload == "ingest" and args.ingest_segment:
        per_gpu = int(round(args.ingest_tib * (1 << 40) / (4 << 20) / 8 * args.ingest_scale))
        pool = min(args.ingest_batch, per_gpu) * args.ingest_segment  # distinct bytes for one launch, no aliasing
    data = torch.empty(pool, dtype=torch.uint8, device=device)
    ctx.fill_synthetic(data.data_ptr(), pool, seed, stream.cuda_stream)
    if args.workload == "mixed":
        sizes, offs = mixed_geometry(args.mixed_chunks, pool, 7 + rank)  # longest first
        L = max(1, args.mixed_launches)
        batches = [DeviceBatch(data.data_ptr(), offs[k::L], sizes[k::L], **kw) for k in range(L)]
        total = int(sizes.sum())
        return data, batches, [int(sizes[k::L].sum()) for k in range(L)], {
            "workload": f"mixed ChunkSize 64K..64M x {args.mixed_chunks} chunks (BASELINE configs[3]) at random "
                        f"offsets of a {args.pool_gib} GiB pool",
            "chunks_per_gpu": args.mixed_chunks, "bytes_per_gpu": total, "pool_bytes": pool, "launches": L}
    chunk = 4 << 20
    per_gpu = int(round(args.ingest_tib * (1 << 40) / chunk / 8 * args.ingest_scale))
    if args.ingest_segment:
        # Distinct data in every launch: 196 608 x 4 MiB cannot be resident at once (768 GiB), so each
        # chunk arrives as 4 MiB / segment Writes -- the per-PATCH resume of filereceiver.go:182-226,
        # as efes_hash_host streams host chunks -- with the states resident in HBM between launches.
        # Launch (g, s) hashes segment s of the chunks of group g from a buffer of
        # ingest_batch x segment distinct bytes (re-filled by the "network" between segments in a
        # real ingest; here the same bytes, so chunk j is its 1 MiB repeated), one job per chunk.
        seg = args.ingest_segment
        nseg = chunk // seg
        batches, nbytes = [], []
        for start in range(0, per_gpu, args.ingest_batch):
            m = min(args.ingest_batch, per_gpu - start)
            base = DeviceBatch(data.data_ptr(), np.arange(m, dtype=np.uint64) * np.uint64(seg), np.full(m, seg),
                               **dict(kw, fresh=False))
            for k in range(nseg):
                batches.append(base.variant(fresh=k == 0, finalize=k == nseg - 1))
                nbytes.append(m * seg)
        return data, batches, nbytes, {
            "workload": f"{args.ingest_tib:g} TiB ingest over 8 GPUs, this GPU's share x{args.ingest_scale:g} "
                        f"(BASELINE configs[4]): 4 MiB chunks as {nseg} x {seg >> 20} MiB segment Writes, distinct "
                        f"bytes in every launch",
            "chunks_per_gpu": per_gpu, "chunk_bytes": chunk, "segment_bytes": seg, "launches": len(batches),
            "distinct_bytes_per_launch": min(args.ingest_batch, per_gpu) * seg}
    slots = pool // chunk
    batches, nbytes = [], []
    for start in range(0, per_gpu, args.ingest_batch):
        m = min(args.ingest_batch, per_gpu - start)
        idx = (np.arange(start, start + m, dtype=np.uint64) + np.uint64(rank * 7919)) % np.uint64(slots)
        batches.append(DeviceBatch(data.data_ptr(), idx * np.uint64(chunk), np.full(m, chunk), **kw))
        nbytes.append(m * chunk)
    return data, batches, nbytes, {"workload": f"{args.ingest_tib:g} TiB ingest over 8 GPUs, this GPU's share "
                                               f"x{args.ingest_scale:g} (BASELINE configs[4]), chunks aliasing a "
                                               f"{args.pool_gib} GiB pool",
                                   "chunks_per_gpu": per_gpu, "chunk_bytes": chunk, "pool_bytes": pool,
                                   "launches": len(batches)}


# Instruction-issue ceilings (DESIGN_NOTES.md §4-5): a wave64 integer VALU instruction holds its SIMD
# for 4 cycles (SQ_INSTS_VALU == SQ_ACTIVE_INST_VALU quad-cycles in profiles/r01_pmc), and
#   DEEP: one message per wave; its SHA-1 chain is 405 VALU per 64-B block (80 rounds x 5 + 5);
#   WIDE: one message per lane; VALU per 64-B block per wave from SQ_INSTS_VALU of a configs[4]-sized
#         launch: WIDE_VALU_FUSED (SHA-1 rounds + schedule, 16 byte swaps, 97 CRC-32 ops from the
#         position tables, loop; 712.4 with round 5's pacing every 32 blocks, profiles/r05_clock/clock2.txt;
#         715.0 with round 4's whole-line loads, 716.5 in round 3, 725 with slicing-by-8) and WIDE_VALU_SHA1
#         (SHA-1 only: 613.8, profiles/r03_wide_pmc/sha1_only_summary.txt, 1.23552e11 / (3 072 waves x 65 536 blocks)).
WIDE_VALU_FUSED = 712.4
WIDE_VALU_SHA1 = 613.8
CLOCK_HZ = 2.4e9
N_SIMD = 1024
VALU_CYC = 4


SMI_JOIN_S = 2.0  # bound on waiting for the amdsmi poll thread (it polls every 2 ms)
_SMI_STATE = {"module": None, "tried": False, "stuck": False}


def _smi_module():
    """amdsmi, initialised ONCE per process (amdsmi_shut_down registered at exit), or None when it
    is absent or refuses.  Every ClockMeter shares it."""
    import atexit

    if not _SMI_STATE["tried"]:
        _SMI_STATE["tried"] = True
        try:
            import amdsmi

            amdsmi.amdsmi_init()
        except Exception:  # noqa: BLE001 -- amdsmi absent or refused: the probe alone
            return None
        _SMI_STATE["module"] = amdsmi

        def _shut_down():
            if not _SMI_STATE["stuck"]:  # a poll thread still inside amdsmi: leave the library alone
                try:
                    amdsmi.amdsmi_shut_down()
                except Exception:  # noqa: BLE001
                    pass

        atexit.register(_shut_down)
    return _SMI_STATE["module"]


class ClockMeter:
    """The effective engine clock over a timed region (the VALU-issue ceilings scale with it), read two
    ways at once:
      probe -- two marker launches on the measured stream (tools/clockprobe.hip) bracket the region;
               each records s_memtime (shader clock) and s_memrealtime (100 MHz) per CU, matched by
               CU (memtime counters of different units have different offsets), median over CUs;
      smi   -- amdsmi's per-XCD current_gfxclk, polled every 2 ms by a host thread, averaged.
    Calibrated against GRBM_GUI_ACTIVE / 8 / ns of the same kernels (profiles/r05_clock/): `mhz` is
    the probe's (within 1 %), the amdsmi mean only when the probe library is missing.  amdsmi is
    initialised once per process (_smi_module) and the poll thread's join is bounded (SMI_JOIN_S):
    neither half can hold the bench (DESIGN_NOTES.md "The r05_check hang")."""

    def __init__(self, dev_index: int):
        import ctypes

        self.dev = dev_index
        self.probe = None
        self.smi = None
        path = os.path.join(ROOT, "tools", "libclockprobe.so")
        bdf = None
        if os.path.exists(path):
            try:
                self.probe = ctypes.CDLL(path)
                self.probe.clockprobe_mark.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
                self.probe.clockprobe_read.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                                       ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)]
                buf = ctypes.create_string_buffer(64)
                if self.probe.clockprobe_pci_bus_id(dev_index, buf, 64) == 0:
                    bdf = buf.value.decode().lower()
            except (OSError, AttributeError):
                self.probe = None
        self.bdf = bdf
        amdsmi = _smi_module()
        try:
            if amdsmi is not None:
                handles = amdsmi.amdsmi_get_processor_handles()
                pick = handles[dev_index] if dev_index < len(handles) else None
                for h in handles:
                    if bdf and str(amdsmi.amdsmi_get_gpu_device_bdf(h)).lower() == bdf:
                        pick = h
                if pick is not None:
                    amdsmi.amdsmi_get_gpu_metrics_info(pick)
                    self.smi = (amdsmi, pick)
        except Exception:  # noqa: BLE001 -- amdsmi refused: the probe alone
            self.smi = None
        self._thread = None
        self._samples = []
        self._stop = None
        self._marked = False
        self.smi_dropped = None

    def _poll(self, stop, samples):
        amdsmi, h = self.smi
        while not stop.is_set():
            try:
                m = amdsmi.amdsmi_get_gpu_metrics_info(h)
                v = [float(x) for x in m.get("current_gfxclks", []) if isinstance(x, (int, float)) and 0 < x < 65535]
                if v:
                    samples.append(sum(v) / len(v))
            except Exception:  # noqa: BLE001
                return
            stop.wait(0.002)

    def start(self, stream: int):
        """Before the region's first launch on `stream` (a hipStream_t handle)."""
        import threading

        self._samples, self._stop = [], threading.Event()
        self._marked = self.probe is not None and self.probe.clockprobe_mark(self.dev, stream, 0) == 0
        if self.smi:
            self._thread = threading.Thread(target=self._poll, args=(self._stop, self._samples), daemon=True,
                                            name="clock-smi-poll")
            self._thread.start()

    def end(self, stream: int):
        """After the region's last launch on `stream`, before the caller synchronizes."""
        if self._marked:
            self._marked = self.probe.clockprobe_mark(self.dev, stream, 1) == 0

    def stop(self) -> dict:
        """After the caller synchronized the stream."""
        import ctypes

        out = {"unit": "MHz"}
        if self._marked:
            mhz, sec, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
            if self.probe.clockprobe_read(self.dev, ctypes.byref(mhz), ctypes.byref(sec), ctypes.byref(n)) == 0:
                out.update({"probe_mhz": round(mhz.value, 1), "probe_seconds": round(sec.value, 4),
                            "probe_cus": n.value})
        if self._thread:
            self._stop.set()
            self._thread.join(SMI_JOIN_S)
            if self._thread.is_alive():
                # an amdsmi call that does not return must not hold the bench: the thread is a
                # daemon, this meter stops using amdsmi for the rest of the process, and the
                # process-wide amdsmi_shut_down at exit is skipped (DESIGN_NOTES.md "r05_check hang")
                _SMI_STATE["stuck"] = True
                self.smi, self.smi_dropped = None, f"amdsmi poll did not return within {SMI_JOIN_S} s; dropped"
                self._samples = []
            self._thread = None
            if self.smi_dropped:
                out["smi_note"] = self.smi_dropped
            elif self._samples:
                s = sorted(self._samples)
                out.update({"smi_mhz_mean": round(sum(s) / len(s), 1), "smi_mhz_min": round(s[0], 1),
                            "smi_mhz_max": round(s[-1], 1), "smi_samples": len(s)})
                if len(s) < 25:  # amdsmi's clock lags its window: a region of a few ms reads the clock before it
                    out["smi_note"] = ("fewer than 25 samples over the region: amdsmi's reading lags and is not "
                                       "this region's clock (span leg: profiles/r05_span_clock/summary.txt)")
        # the probe: within 0.1-1 % of GRBM_GUI_ACTIVE in the same run; the amdsmi mean strays by up to
        # 6 % (it samples clock transients between launches; profiles/r05_clock/calibration.txt)
        out["mhz"] = out.get("probe_mhz", out.get("smi_mhz_mean"))
        return out


_CLOCK = None


def clock_meter(dev_index: int):
    global _CLOCK
    if _CLOCK is None or _CLOCK.dev != dev_index:
        _CLOCK = ClockMeter(dev_index)
    return _CLOCK


def binding_roofline(kernel: str, achieved_gbs: float, concurrent_msgs: int, sha1_only: bool, clock=None):
    if kernel == "deep_kernel":
        ceiling = min(concurrent_msgs, N_SIMD) * 64 * CLOCK_HZ / (405 * VALU_CYC) / 1e9
        model = ("serial SHA-1 chain: each of min(messages, 1024 SIMDs) messages advances one 64-B block per "
                 "405 VALU x 4 cycles at 2.4 GHz (one wave per message)")
    else:
        per_block = WIDE_VALU_SHA1 if sha1_only else WIDE_VALU_FUSED
        lanes = min(concurrent_msgs, N_SIMD * 64 * 8)
        ceiling = min(lanes / 64, N_SIMD) * 64 * 64 * CLOCK_HZ / (per_block * VALU_CYC) / 1e9
        model = (f"VALU issue: {per_block} VALU per 64-B block per wave of 64 messages, 4 cycles each, "
                 "every SIMD busy at 2.4 GHz")
    out = {"bound": "valu-issue", "achieved": round(achieved_gbs, 2), "ceiling": round(ceiling, 2), "unit": "GB/s",
           "frac": round(achieved_gbs / ceiling, 4), "model": model}
    mhz = (clock or {}).get("mhz")
    if mhz:  # the same ceiling at the clock the region actually ran at
        at = ceiling * mhz * 1e6 / CLOCK_HZ
        out.update({"clock_mhz": mhz, "ceiling_at_clock": round(at, 2), "frac_at_clock": round(achieved_gbs / at, 4)})
    return out


def run_timed(batches, steps: int, warmup: int, mode: int, device: str, stream, dist, progress: bool = False):
    """W untimed warm-up launches, then exactly `steps` launches bracketed by barrier +
    synchronize; returns (wall seconds of this rank, average kernel ms from HIP events recorded
    on the launch stream, the effective engine clock over the timed launches (ClockMeter))."""
    import torch

    for _ in range(warmup):
        batches[0].submit(mode)
    torch.cuda.synchronize(device)
    if warmup:
        assert (batches[0].status_host() == 0).all(), "hash jobs reported an error status"
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(device)
    clk = clock_meter(torch.device(device).index or 0)
    clk.start(stream.cuda_stream)
    t0 = time.perf_counter()
    ev0.record(stream)
    for k in range(steps):
        batches[k % len(batches)].submit(mode)
        if progress:
            torch.cuda.synchronize(device)
            print(f"[bench] step {k + 1}/{steps} done at {time.perf_counter() - t0:.1f} s", file=sys.stderr,
                  flush=True)
    ev1.record(stream)
    clk.end(stream.cuda_stream)
    torch.cuda.synchronize(device)
    if dist:
        dist.barrier()
    wall = time.perf_counter() - t0
    clock = clk.stop()
    for b in batches:
        assert (b.status_host() == 0).all(), "hash jobs reported an error status"
    return wall, ev0.elapsed_time(ev1) / max(1, steps), clock


def ingest_leg(args, rank: int, world: int, ctx, device: str, stream, mode: int, dist=None):
    """BASELINE configs[4] beside the metric: this GPU's share of a 10 TiB ingest of 4 MiB
    chunks (327 680 chunks, per-GPU queue) in launches of 196 608 chunks aliasing a 64 GiB pool.
    At N > 1 every rank hashes its own share (weak scaling, no data-path collective): the launches
    are bracketed by a barrier + synchronize on every rank, the wall time is the max over ranks and
    the value is the bytes of ALL ranks over it (the north_star's 10 TiB over 8 GPUs at N = 8)."""
    import argparse as _ap

    import torch

    a = _ap.Namespace(**vars(args))
    # launches of 196 608 chunks = 3 resident WIDE waves on every SIMD (then the remainder):
    # 2 613-2 673 GiB/s against 2 395-2 443 for launches of 131 072 (2 waves per SIMD) and 2 408 for one
    # launch of all 327 680 (profiles/r01_sweeps/ingest_batch_*.json)
    a.workload, a.ingest_batch, a.ingest_scale = "ingest", 196608, args.ingest_scale
    with torch.cuda.stream(stream):
        data, batches, step_bytes, config = make_workload(a, rank, world, ctx, device, stream)
        wall, kernel_ms, clock = run_timed(batches, len(batches), 1, mode, device, stream, dist)
        ok = ingest_spot_check(data, batches, config)
    from efes_amd.shard import max_over_ranks

    wall = max_over_ranks(wall, device if args.dist_backend == "nccl" else None)
    total = sum(step_bytes)
    per_launch = total / len(batches)
    achieved = per_launch / (kernel_ms * 1e-3) / 1e9
    per_launch_jobs = batches[0].n
    del data, batches
    torch.cuda.empty_cache()
    # HBM bytes per algorithmic byte of a WIDE launch of this geometry (196 608 distinct 1 MiB
    # messages), FETCH_SIZE x 2 -- calibrated for WIDE's per-lane access pattern on a known byte count
    # (tools/microbench/mb_wide_fetch, profiles/r04_fetch/) -- applied to this leg's average launch
    t = load_traffic("wide_kernel", f"196608x{1 << 20}:sha1+crc32")
    ratio = None if t is None else t / (196608 * (1 << 20))
    return {"value": round(world * total / wall / GiB, 3), "unit": "GiB/s", "n_gpus": world,
            "scaling": "weak", "bytes_per_gpu": total, "max_rank_wall_s": round(wall, 4), "digests_spot_check": ok,
            "workload": config["workload"],
            "chunks": config["chunks_per_gpu"], "launches": config["launches"], "kernel": "wide_kernel",
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 5), "kernel_ms": round(kernel_ms, 3),
                         "traffic": None if ratio is None else round(ratio * per_launch),
                         "traffic_per_algorithmic_byte": None if ratio is None else round(ratio, 4),
                         "algorithmic_bytes_per_launch": int(per_launch)},
            "binding_roofline": binding_roofline("wide_kernel", achieved, per_launch_jobs, args.sha1_only, clock),
            "clock": clock,
            "note": "many concurrent chunks per GPU (configs[4] per-GPU queue); value = all ranks' bytes / the "
                    "slowest rank's wall time; roofline = this rank's kernel; not the headline `value`"}


def sha1_only_leg(args, ctx, data, fused, device: str, stream):
    """BASELINE configs[1] beside the metric: the same 1024 x 4 MiB device-resident chunks, SHA-1
    only (jobs without a CRC-32 state, sha1.go alone), K timed launches like the headline, with
    its own roofline; digests checked against the fused run's."""
    import numpy as np
    import torch

    from efes_amd import MODE_AUTO
    from efes_amd._lib import lib
    from efes_amd.batch import DeviceBatch

    n, chunk = args.chunks, args.chunk_bytes
    with torch.cuda.stream(stream):
        b = DeviceBatch(data.data_ptr(), np.arange(n, dtype=np.uint64) * chunk, np.full(n, chunk), crc32=False,
                        fresh=True, ctx=ctx, device=device)
        wall, kernel_ms, clock = run_timed([b], args.steps, 1, MODE_AUTO, device, stream, None)
    kernel = kernel_names()[lib().efes_auto_mode(ctx.handle, n)]
    achieved = n * chunk / (kernel_ms * 1e-3) / 1e9
    ok = b.sha1_hex() == fused.sha1_hex() and bool((b.sums_host()[:, 20:] == 0).all())
    return {"value": round(args.steps * n * chunk / wall / GiB, 3), "unit": "GiB/s",
            "workload": f"{n} x {chunk >> 20} MiB chunks, SHA-1 only (BASELINE configs[1])", "kernel": kernel,
            "steps": args.steps, "ms_per_step": round(wall * 1e3 / args.steps, 4),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 5), "kernel_ms": round(kernel_ms, 4),
                         "traffic": load_traffic(kernel, f"{n}x{chunk}:sha1")},
            "binding_roofline": binding_roofline(kernel, achieved, n, True, clock)
            if kernel in ("deep_kernel", "wide_kernel") else None, "clock": clock,
            "digests_match_fused_sha1": ok, "note": "same chunks as the metric, SHA-1 only; not `value`"}


def device_bdf(dev_index: int):
    """The PCI address of HIP device `dev_index` ("0000:05:00.0"; the clock probe's
    hipDeviceGetPCIBusId, else torch's device properties), or None."""
    import ctypes

    path = os.path.join(ROOT, "tools", "libclockprobe.so")
    if os.path.exists(path):
        try:
            buf = ctypes.create_string_buffer(64)
            if ctypes.CDLL(path).clockprobe_pci_bus_id(dev_index, buf, 64) == 0 and buf.value:
                return buf.value.decode().lower()
        except (OSError, AttributeError):
            pass
    try:
        import torch

        p = torch.cuda.get_device_properties(dev_index)
        return f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    except Exception:  # noqa: BLE001
        return None


def rank_spot_check(args, data, batches, config) -> bool:
    """hashlib/zlib of the first and last job of this rank's (first) batch against its Sums: the
    headline's chunks and the mixed sizes directly, the segmented ingest through ingest_spot_check."""
    import hashlib
    import zlib

    if config.get("segment_bytes"):
        return ingest_spot_check(data, batches, config)
    b = batches[0]
    if not b.n:
        return True
    ok = bool((b.status_host() == 0).all())
    sums = b.sums_host()
    base = data.data_ptr()
    for j in sorted({0, b.n - 1}):
        off, n = int(b.jobs_host["data"][j]) - base, int(b.jobs_host["length"][j])
        piece = data[off:off + n].cpu().numpy().tobytes()
        ok = ok and bytes(sums[j][:20]) == hashlib.sha1(piece).digest()
        if not args.sha1_only:
            ok = ok and int.from_bytes(bytes(sums[j][20:24]), "big") == zlib.crc32(piece)
    return bool(ok)


def ingest_spot_check(data, batches, config) -> bool:
    """hashlib/zlib of two chunks per launch group against the Sums of the segmented ingest (chunk j
    of a group = its segment's bytes, once per segment); True when the leg is not segmented."""
    import hashlib
    import zlib

    seg = config.get("segment_bytes")
    if not seg:
        return True
    nseg = config["chunk_bytes"] // seg
    ok = True
    for g in range(0, len(batches), nseg):
        last = batches[g + nseg - 1]
        for j in (0, last.n - 1):
            piece = data[j * seg:(j + 1) * seg].cpu().numpy().tobytes()
            chunk = piece * nseg
            s = last.sums_host()[j]
            ok = ok and bytes(s[:20]) == hashlib.sha1(chunk).digest() and \
                int.from_bytes(bytes(s[20:24]), "big") == zlib.crc32(chunk)
    return bool(ok)


def concurrency_leg(args, ctx, device: str, stream):
    """How the rate of 4 MiB chunks depends on how many are in flight (DESIGN_NOTES.md §4): one AUTO
    launch per count (DEEP up to one chunk per SIMD, FED4 / FED4E up to 32 / 48 per CU, GROUP4,
    then WIDE) over distinct bytes: up to 16 384 chunks (64 GiB) whole, beyond that each chunk as
    four 1 MiB segment Writes with the states resident (as the configs[4] leg), since 4 MiB x 65 536
    does not fit in HBM -- aliased chunks would be served from the caches.  One warm-up and two
    timed passes per point."""
    import numpy as np
    import torch

    from efes_amd._lib import MODE_AUTO, lib
    from efes_amd.batch import DeviceBatch

    names = kernel_names()
    chunk, seg = 4 << 20, 1 << 20
    points = []
    with torch.cuda.stream(stream):
        for n in (1024, 2048, 4096, 8192, 16384, 65536, 196608):
            whole = n * chunk <= 64 << 30
            piece = chunk if whole else seg
            data = torch.empty(n * piece, dtype=torch.uint8, device=device)
            ctx.fill_synthetic(data.data_ptr(), n * piece, 0xC0C0, stream.cuda_stream)
            offs = np.arange(n, dtype=np.uint64) * np.uint64(piece)
            if whole:
                batches = [DeviceBatch(data.data_ptr(), offs, np.full(n, chunk), fresh=True, ctx=ctx, device=device)]
            else:
                base = DeviceBatch(data.data_ptr(), offs, np.full(n, seg), ctx=ctx, device=device)
                batches = [base.variant(fresh=k == 0, finalize=k == 3) for k in range(4)]
            wall, kernel_ms, clock = run_timed(batches, 2 * len(batches), 1, MODE_AUTO, device, stream, None)
            points.append({"chunks": n, "kernel": names[lib().efes_auto_mode(ctx.handle, n)],
                           "segments": len(batches), "GiB/s": round(2 * n * chunk / wall / GiB, 1),
                           "ms_per_launch": round(kernel_ms, 2), "clock_mhz": clock.get("mhz")})
            del batches, data
            torch.cuda.empty_cache()
    return {"unit": "GiB/s", "chunk_bytes": chunk, "points": points,
            "note": "n fresh 4 MiB chunks (fused SHA-1+CRC32), AUTO shape, distinct bytes (segments = 1 MiB Writes "
                    "per chunk when n x 4 MiB exceeds 64 GiB); not `value`"}


def mixed_leg(args, rank: int, world: int, ctx, device: str, stream):
    """BASELINE configs[3] beside the metric: 65 536 chunks of the eleven ChunkSize values
    64K..64M (752 GiB, at random offsets of a 200 GiB pool), placed by efes_plan_batch (grouped-DEEP parts
    on CUs of their own, concurrent with WIDE); one warm-up and one timed step."""
    import argparse as _ap

    import torch

    from efes_amd.batch import MODE_PLAN

    a = _ap.Namespace(**vars(args))
    a.workload = "mixed"
    # 752 GiB of chunks at random offsets of a 200 GiB pool (3.8 chunks over each byte): the 64 GiB
    # pool of rounds 1-3 (12 over each byte) measured the same, 856.9-858.1 vs 856.7-858.5 GiB/s in
    # three interleaved pairs (profiles/r04_mixed_pool/ab.log) -- the 64 MiB chains set the makespan
    a.pool_gib = max(args.pool_gib, 200)
    with torch.cuda.stream(stream):
        data, batches, step_bytes, config = make_workload(a, rank, world, ctx, device, stream)
        for b in batches:
            b.make_plan()
        wall, kernel_ms, clock = run_timed(batches, len(batches), 1, MODE_PLAN, device, stream, None)
    total = sum(step_bytes)
    names = kernel_names()
    parts = [{"jobs": j, "kernel": names[m], "exclusive_cus": x} for j, m, x in batches[0].plan.parts()]
    achieved = total / len(batches) / (kernel_ms * 1e-3) / 1e9
    del data, batches
    torch.cuda.empty_cache()
    return {"value": round(total / wall / GiB, 3), "unit": "GiB/s", "workload": config["workload"],
            "chunks": config["chunks_per_gpu"], "bytes": total, "plan": parts,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 5), "kernel_ms": round(kernel_ms, 3)},
            "clock": clock, "note": "makespan set by the 64 MiB chunks' SHA-1 chains (DESIGN_NOTES.md §4 batch planner); not `value`"}


def read_ceiling(data, n: int, device: str, stream, reps: int = 3):
    """The read ceiling of the span leg's own buffer: a pure LDS-DMA nontemporal read of it in the
    span kernel's shape (tools/readprobe.hip), timed with HIP events on the leg's stream.  The span
    CRC's rate follows the buffer's allocation, so its fraction is also reported
    against this."""
    import ctypes

    import torch

    path = os.path.join(ROOT, "tools", "libreadprobe.so")
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    lib.readprobe_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
    dev = torch.device(device).index or 0
    groups = torch.cuda.get_device_properties(dev).multi_processor_count
    usable = n - n % (64 << 10)
    if lib.readprobe_launch(dev, data.data_ptr(), usable, groups, stream.cuda_stream) != 0:  # warm-up
        return None
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        lib.readprobe_launch(dev, data.data_ptr(), usable, groups, stream.cuda_stream)
    e1.record(stream)
    stream.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return {"value": round(usable / (ms * 1e-3) / 1e9, 1), "unit": "GB/s",
            "kind": "LDS-DMA nontemporal read of the same buffer, the span kernel's shape (tools/readprobe.hip)",
            "microbenchmark": "7.0-7.2 TB/s on a fresh buffer (tools/microbench/mb_glds, profiles/r05_span_nt/)"}


def span_crc_leg(args, ctx, device: str, stream, gib: int = 16, reps: int = 5):
    """CRC-32 alone of ONE object resident in HBM (efes_crc32_span, segment-
    parallel over all CUs), against the HBM roofline; the first GiB is checked against zlib, and the
    oracle's serial crc32.go restatement is timed on one host core over that GiB."""
    import zlib

    import torch

    from oracle import oracle

    n = gib << 30
    with torch.cuda.stream(stream):
        data = torch.empty(n, dtype=torch.uint8, device=device)
        ctx.fill_synthetic(data.data_ptr(), n, 0x5BA4, stream.cuda_stream)
        st = torch.zeros(1, dtype=torch.int64, device=device)
        ctx.crc32_span(data.data_ptr(), n, st.data_ptr(), stream.cuda_stream)  # warm-up
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        stream.synchronize()
        clk = clock_meter(torch.device(device).index or 0)
        clk.start(stream.cuda_stream)
        e0.record(stream)
        for _ in range(reps):
            st.zero_()
            ctx.crc32_span(data.data_ptr(), n, st.data_ptr(), stream.cuda_stream)
        e1.record(stream)
        clk.end(stream.cuda_stream)
        stream.synchronize()
        clock = clk.stop()
        ms = e0.elapsed_time(e1) / reps
        ceiling = read_ceiling(data, n, device, stream)
        st.zero_()
        ctx.crc32_span(data.data_ptr(), 1 << 30, st.data_ptr(), stream.cuda_stream)
        stream.synchronize()
        head = data[: 1 << 30].cpu().numpy()
    ok = (int(st.item()) & 0xFFFFFFFF) == zlib.crc32(head)
    o = oracle.Crc32()
    t0 = time.perf_counter()
    o.write(head)
    cpu_s = time.perf_counter() - t0
    ok = ok and o.sum32() == zlib.crc32(head)
    del data, head
    torch.cuda.empty_cache()
    achieved = n / (ms * 1e-3) / 1e9
    return {"workload": f"one {gib} GiB object, CRC-32 only (efes_crc32_span)", "bytes": n,
            "value": round(n / (ms * 1e-3) / GiB, 1), "unit": "GiB/s", "kernel": "span_kernel",
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 4), "ms_per_call": round(ms, 3),
                         "traffic": load_traffic("span_kernel", f"{gib}GiB:span"),
                         "read_ceiling": ceiling,
                         "frac_of_read_ceiling": None if not ceiling else round(achieved / ceiling["value"], 4)},
            "cpu_port_1core": {"value": round((1 << 30) / cpu_s / GiB, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
                               "sample": "oracle crc32digest.Write (slicing-by-8, crc32.go:153-169) over the first GiB"},
            "crc_matches_zlib": ok, "clock": clock, "note": "HIP events on the launch stream; not `value`"}


def main(argv=None):
    args = parse_args(argv)
    if args.watchdog > 0:
        import faulthandler

        faulthandler.dump_traceback_later(args.watchdog, exit=False)  # all threads' stacks to stderr
    legs = Legs()
    import torch

    from efes_amd import MODE_AUTO, MODE_DEEP, MODE_WIDE
    from efes_amd._lib import MODE_FED4, MODE_FED4E, MODE_GROUP, lib
    from efes_amd.batch import MODE_PLAN
    from efes_amd.hashing import default_context
    from efes_amd.shard import env_rank, max_over_ranks

    rank, local, world = env_rank()
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)
    dev_index = 0 if args.all_ranks_on_device0 else local
    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(dev_index)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        else:
            dist.init_process_group(args.dist_backend)
    device = f"cuda:{dev_index}"
    torch.cuda.set_device(dev_index)
    ctx = default_context(dev_index)
    stream = torch.cuda.Stream(device=device)
    modes = {"auto": MODE_AUTO, "deep": MODE_DEEP, "wide": MODE_WIDE, "plan": MODE_PLAN}
    modes.update({f"group{g}": v for g, v in MODE_GROUP.items()})
    modes["fed4"], modes["fed4e"] = MODE_FED4, MODE_FED4E
    mode = modes["plan" if args.mode == "auto" and args.workload == "mixed" else args.mode]

    if args.workload == "uploads":
        res = uploads_workload(args, ctx)
        if rank == 0:
            print(json.dumps({"metric": "GiB/s hashed through concurrent uploads (efes_queue), host-resident",
                              "workload": "uploads", **res}), flush=True)
        if dist:
            dist.destroy_process_group()
        return
    print(f"[bench] headline ({args.workload}): start", file=sys.stderr, flush=True)
    with torch.cuda.stream(stream):
        data, batches, step_bytes, config = make_workload(args, rank, world, ctx, device, stream)
        if mode == MODE_PLAN:
            for b in batches:
                b.make_plan()  # host-side planning stays outside the timed region
        steps = args.steps if len(batches) == 1 else len(batches)
        wall, kernel_ms, clock = run_timed(batches, steps, args.warmup, mode, device, stream, dist, args.progress)
    print(f"[bench] headline: {steps} steps in {wall:.3f} s on this rank", file=sys.stderr, flush=True)
    rank_wall = wall
    wall = max_over_ranks(wall, device if args.dist_backend == "nccl" else None)  # slowest rank

    bytes_timed = sum(step_bytes[k % len(step_bytes)] for k in range(steps))
    value = world * bytes_timed / wall / GiB
    njobs = batches[0].n
    launched = lib().efes_auto_mode(ctx.handle, njobs) if mode == MODE_AUTO else mode
    kernel_name = kernel_names().get(launched, "planned parts")  # MODE_PLAN: named from the plan below
    plan = None
    if mode == MODE_PLAN:
        p0 = batches[0].plan
        names = kernel_names()
        plan = {"parts": [{"jobs": j, "kernel": names[m], "exclusive_cus": x} for j, m, x in p0.parts()],
                "model_seconds": round(p0.est_seconds, 4)}
        kernel_name = " + ".join(p["kernel"] for p in plan["parts"]) + " (concurrent streams)"
    per_launch = bytes_timed / steps
    workload_key = f"{config['workload']}:{'sha1' if args.sha1_only else 'sha1+crc32'}"
    if args.workload == "chunks4m":
        workload_key = f"{njobs}x{args.chunk_bytes}:{'sha1' if args.sha1_only else 'sha1+crc32'}"
    achieved = per_launch / (kernel_ms * 1e-3) / 1e9
    config.update({"kernel": kernel_name, "parallelism": f"per-GPU queues x{world}, no collectives"})
    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall * 1e3 / steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (device-generated splitmix64 bytes)",
        "config": config,
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 5),
            "traffic": load_traffic(kernel_name, workload_key),
            "kernel_ms": round(kernel_ms, 4),
            "algorithmic_bytes_per_launch": int(per_launch),
        },
        "binding_roofline": (binding_roofline(kernel_name, achieved, njobs, args.sha1_only, clock)
                             if kernel_name in ("deep_kernel", "wide_kernel") else None),
        "clock": clock,
        "cpu_baseline": None,
    }
    if plan:
        out["config"]["plan"] = plan
    # Which device each rank ran on, its own rate and kernel time, and spot checks of its digests
    # (SURVEY.md §8(e)): a weak-scaling line must show N distinct GPUs doing the work.  After the timed
    # region; one all_gather_object of a small dict, measurement only.
    from efes_amd.shard import gather_rank_records, summarize_ranks

    rec = {"rank": rank, "local_rank": local, "device": dev_index, "bdf": device_bdf(dev_index),
           "GiB/s": round(bytes_timed / rank_wall / GiB, 3), "wall_s": round(rank_wall, 4),
           "kernel_ms": round(kernel_ms, 4), "clock_mhz": clock.get("mhz"),
           "spot_check": rank_spot_check(args, data, batches, config)}
    records = gather_rank_records(rec)
    out["ranks"] = records
    out["ranks_check"] = summarize_ranks(records, world, args.all_ranks_on_device0)
    if args.workload == "chunks4m":
        n, chunk = args.chunks, args.chunk_bytes
        if args.host_inclusive == "on" or (args.host_inclusive == "auto" and world == 1):
            out["host_inclusive"] = legs.run("host_inclusive", host_inclusive, ctx, data, n, chunk, not args.sha1_only,
                                                   args.segment_bytes, batches[0])
        if not args.sha1_only and (args.sha1_leg == "on" or (args.sha1_leg == "auto" and world == 1)):
            out["sha1_only_config"] = legs.run("sha1_only_config", sha1_only_leg, args, ctx, data, batches[0], device, stream)
        # the span CRC before the legs that allocate and free 64-200 GiB pools: its rate follows where its
        # buffer lands (a 16 GiB buffer allocated after the mixed leg's 200 GiB pool read 5.8-6.0 TB/s
        # where a fresh one read 6.6; DESIGN.md §4 "Span CRC"), and a standalone caller's buffer is fresh
        if args.span_leg == "on" or (args.span_leg == "auto" and world == 1):
            out["span_crc"] = legs.run("span_crc", span_crc_leg, args, ctx, device, stream)
        if args.ingest_leg in ("on", "auto"):
            out["ingest_config"] = legs.run("ingest_config", ingest_leg, args, rank, world, ctx, device, stream, MODE_AUTO,
                                            dist)
        if args.uploads_leg == "on" or (args.uploads_leg == "auto" and world == 1):
            a = argparse.Namespace(**vars(args))
            a.upload_threads, a.uploads, a.open_per_thread, a.upload_bytes = 32, 8192, 256, 4 << 20
            out["uploads_path"] = legs.run("uploads_path", uploads_workload, a, ctx)
        if args.go_surface_leg == "on" or (args.go_surface_leg == "auto" and world == 1):
            out["go_surface_path"] = legs.run("go_surface_path", go_surface_leg, out.get("uploads_path"))
        if args.latency_leg == "on" or (args.latency_leg == "auto" and world == 1):
            out["patch_latency"] = legs.run("patch_latency", patch_latency_leg, _ints(args.latency_uploads))
        if args.receiver_leg == "on" or (args.receiver_leg == "auto" and world == 1):
            out["receiver_path"] = legs.run("receiver_path", receiver_leg)
        if args.drain_leg == "on" or (args.drain_leg == "auto" and world == 1):
            out["drain_path"] = legs.run("drain_path", drain_leg, _ints(args.drain_workers))
        if args.concurrency_leg == "on" or (args.concurrency_leg == "auto" and world == 1):
            out["concurrency"] = legs.run("concurrency", concurrency_leg, args, ctx, device, stream)
        if args.mixed_leg == "on" or (args.mixed_leg == "auto" and world == 1):
            out["mixed_config"] = legs.run("mixed_config", mixed_leg, args, rank, world, ctx, device, stream)
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            threads = args.cpu_threads or host_threads()
            out["cpu_baseline"] = legs.run("cpu_baseline", cpu_baseline, batches[0], data, min(n, args.cpu_max_chunks), chunk,
                                           threads, not args.sha1_only, args.cpu_seconds)
            out["config0_cpu"] = legs.run("config0_cpu", config0_cpu, data, chunk)
    out["leg_seconds"] = legs.seconds
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()
    if not out["ranks_check"]["ok"]:
        # after the line is out: the driver keeps the measurement, and the run still fails loudly
        print(f"bench.py: rank check failed: {out['ranks_check']}", file=sys.stderr, flush=True)
        sys.exit(3)


if __name__ == "__main__":
    main()
