"""Build libefeshash.so in-tree for gfx950 (hipcc cross-compiles without a GPU).

    python -m efes_amd.build
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB_DIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIB_DIR, "libefeshash.so")
SOURCES = ["efes_kernels.hip", "efes_crc_span.hip", "efes_api.cpp", "efes_ingest.cpp", "efes_queue.cpp", "efes_stream.cpp", "efes_plan.cpp"]
HEADERS = ["efes_internal.hpp", "sha1_device.hpp"]
PUBLIC_HEADERS = ["efes_hash.h", "efes_testing.h"]
ARCH = "gfx950"


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    raise RuntimeError("hipcc not found")


def _stale(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _lib_deps() -> list[str]:
    return ([os.path.join(CSRC, s) for s in SOURCES] + [os.path.join(CSRC, h) for h in HEADERS] +
            [os.path.join(ROOT, "include", h) for h in PUBLIC_HEADERS])


def source_id() -> str:
    """The identity of the library's sources: the first 16 hex digits of a SHA-256 over every source and
    header file (name and bytes, in a fixed order).  Compiled into the library (efes_build_id), so a
    test on the GPU box can tell that the .so it loaded was built from the sources beside it."""
    import hashlib

    h = hashlib.sha256()
    for path in _lib_deps():
        h.update(os.path.relpath(path, ROOT).encode() + b"\0")
        with open(path, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def build_lib(force: bool = False, verbose: bool = False) -> str:
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    deps = _lib_deps()
    if not force and not _stale(LIB, deps):
        return LIB
    os.makedirs(LIB_DIR, exist_ok=True)
    tmp = LIB + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", f'-DEFES_BUILD_ID="{source_id()}"',
           "-I", os.path.join(ROOT, "include"), "-o", tmp] + srcs
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


def build_variant(name: str, defines: list[str]) -> str:
    """An A/B build of the library with extra -D flags: efes_amd/lib/libefeshash_<name>.so (loaded through
    EFES_LIB_OVERRIDE by the tools/gpu_*_ab.sh scripts; never the product)."""
    out = os.path.join(LIB_DIR, f"libefeshash_{name}.so")
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", *[f"-D{d}" for d in defines],
           "-I", os.path.join(ROOT, "include"), "-o", out + ".tmp"] + srcs
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


def build_tools() -> list[str]:
    """Native benchmark drivers under tools/ (link the in-tree library; not part of the product)."""
    out = []
    src = os.path.join(ROOT, "tools", "bench_uploads.cpp")
    exe = os.path.join(ROOT, "tools", "bench_uploads")
    devices_hpp = os.path.join(ROOT, "tools", "efes_devices.hpp")
    if os.path.exists(src) and _stale(exe, [src, LIB, devices_hpp]):
        subprocess.run([hipcc(), "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"), src, "-o", exe,
                        "-L", LIB_DIR, "-lefeshash", "-Wl,-rpath,$ORIGIN/../efes_amd/lib", "-pthread"], check=True)
    if os.path.exists(exe):
        out.append(exe)
    src = os.path.join(ROOT, "tools", "bench_go_surface.cpp")
    exe = os.path.join(ROOT, "tools", "bench_go_surface")
    if os.path.exists(src) and _stale(exe, [src, LIB, os.path.join(ROOT, "include", "efes_hash.h"), devices_hpp]):
        subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Wextra", "-pthread", "-I", os.path.join(ROOT, "include"),
                        src, "-o", exe, "-L", LIB_DIR, "-lefeshash", "-Wl,-rpath,$ORIGIN/../efes_amd/lib"], check=True)
    if os.path.exists(exe):
        out.append(exe)
    src = os.path.join(ROOT, "tools", "clockprobe.hip")  # bench.py's engine-clock probe
    so = os.path.join(ROOT, "tools", "libclockprobe.so")
    if os.path.exists(src) and _stale(so, [src]):
        subprocess.run([hipcc(), f"--offload-arch={ARCH}", "-O2", "-std=c++17", "-fPIC", "-shared", src, "-o", so + ".tmp"],
                       check=True)
        os.replace(so + ".tmp", so)
    if os.path.exists(so):
        out.append(so)
    src = os.path.join(ROOT, "tools", "readprobe.hip")  # bench.py's read ceiling of the span leg's buffer
    so = os.path.join(ROOT, "tools", "libreadprobe.so")
    if os.path.exists(src) and _stale(so, [src]):
        subprocess.run([hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", src, "-o", so + ".tmp"],
                       check=True)
        os.replace(so + ".tmp", so)
    if os.path.exists(so):
        out.append(so)
    src = os.path.join(ROOT, "tools", "bench_receiver.cpp")
    exe = os.path.join(ROOT, "tools", "bench_receiver")
    if os.path.exists(src) and _stale(exe, [src, RECEIVER_LIB, RECEIVER_HDR, LIB]):
        subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Wextra", "-pthread", "-I", os.path.join(ROOT, "include"),
                        src, "-o", exe, "-L", LIB_DIR, "-lefesreceiver", "-lefeshash",
                        "-Wl,-rpath,$ORIGIN/../efes_amd/lib"], check=True)
    if os.path.exists(exe):
        out.append(exe)
    return out


RECEIVER_SRC = os.path.join(HERE, "host", "efes_receiver.cpp")
RECEIVER_HDR = os.path.join(HERE, "host", "efes_receiver.hpp")
RECEIVER_LIB = os.path.join(LIB_DIR, "libefesreceiver.so")


def build_receiver(force: bool = False) -> str:
    """libefesreceiver.so: the C++ mirror of the Go callers above the C ABI (fileinfo.go,
    filereceiver.go, sha1file.go), linked against libefeshash.so."""
    deps = [RECEIVER_SRC, RECEIVER_HDR, LIB, os.path.join(ROOT, "include", "efes_hash.h")]
    if force or _stale(RECEIVER_LIB, deps):
        tmp = RECEIVER_LIB + ".tmp"
        subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Wextra", "-fPIC", "-shared", "-pthread",
                        "-I", os.path.join(ROOT, "include"), RECEIVER_SRC, "-o", tmp,
                        "-L", LIB_DIR, "-lefeshash", "-Wl,-rpath,$ORIGIN"], check=True)
        os.replace(tmp, RECEIVER_LIB)
    return RECEIVER_LIB


def build_receiver_test() -> str:
    """tests/cpp/receiver_test: the reference's receiver / Sha1File tests replayed against the C++
    mirror, checked against the oracle (test infrastructure)."""
    src = os.path.join(ROOT, "tests", "cpp", "receiver_test.cpp")
    exe = os.path.join(ROOT, "tests", "cpp", "receiver_test")
    oracle_lib = os.path.join(ROOT, "oracle", "liboracle.so")
    if os.path.exists(src) and _stale(exe, [src, RECEIVER_LIB, RECEIVER_HDR, LIB, oracle_lib]):
        subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Wextra", "-pthread", "-I", os.path.join(ROOT, "include"),
                        src, "-o", exe, "-L", LIB_DIR, "-lefesreceiver", "-lefeshash",
                        "-L", os.path.join(ROOT, "oracle"), "-loracle",
                        "-Wl,-rpath,$ORIGIN/../../efes_amd/lib", "-Wl,-rpath,$ORIGIN/../../oracle"], check=True)
    return exe


def build_consumer_test() -> str:
    """tests/c/efes_consumer_test: a C consumer of the ABI checked against the oracle (test infrastructure)."""
    src = os.path.join(ROOT, "tests", "c", "efes_consumer_test.c")
    exe = os.path.join(ROOT, "tests", "c", "efes_consumer_test")
    oracle_lib = os.path.join(ROOT, "oracle", "liboracle.so")
    if os.path.exists(src) and _stale(exe, [src, LIB, oracle_lib, os.path.join(ROOT, "include", "efes_hash.h")]):
        subprocess.run(["gcc", "-O2", "-std=c11", "-Wall", "-Wextra", "-pthread", src, "-o", exe,
                        "-L", LIB_DIR, "-lefeshash", "-L", os.path.join(ROOT, "oracle"), "-loracle",
                        "-Wl,-rpath,$ORIGIN/../../efes_amd/lib", "-Wl,-rpath,$ORIGIN/../../oracle"], check=True)
    return exe


def build_lifecycle_test() -> str:
    """tests/c/efes_lifecycle_test_asan: the Go binding's object lifecycle against an AddressSanitizer
    build of the library's host code (tools/asan_build.sh; test infrastructure)."""
    exe = os.path.join(ROOT, "tests", "c", "efes_lifecycle_test_asan")
    srcs = [os.path.join(CSRC, s) for s in SOURCES] + [os.path.join(CSRC, h) for h in HEADERS]
    deps = srcs + [os.path.join(ROOT, "tests", "c", "efes_lifecycle_test.c"), os.path.join(ROOT, "tools", "asan_build.sh"),
                   os.path.join(ROOT, "oracle", "liboracle.so")] + [os.path.join(ROOT, "include", h) for h in PUBLIC_HEADERS]
    if _stale(exe, deps):
        try:
            subprocess.run(["bash", os.path.join(ROOT, "tools", "asan_build.sh")], check=True)
        except (OSError, subprocess.CalledProcessError) as e:
            # test-only artefact: a toolchain without the clang ASan runtime must not fail the product
            # build; tests/test_gpu_lifecycle.py fails on its own when the binary is missing
            print(f"efes_amd.build: the ASan lifecycle test was not built ({e})", file=sys.stderr)
            return None
    return exe


def build_oracle() -> str:
    """The CPU checker (test infrastructure; never linked into the product)."""
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    return os.path.join(ROOT, "oracle", "liboracle.so")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--variant":  # python -m efes_amd.build --variant NAME DEFINE...
        print(build_variant(sys.argv[2], sys.argv[3:]))
        sys.exit(0)
    print(build_lib(force="--force" in sys.argv, verbose=True))
    print(build_tools())
    print(build_oracle())
    print(build_consumer_test())
    print(build_receiver())
    print(build_receiver_test())
    print(build_lifecycle_test())
