"""The C ABI boundary (include/efes_hash.h) without a GPU: exports, layouts, host codecs, tables."""
import ctypes
import os
import re
import subprocess
import zlib

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "efes_hash.h")
HEADERS = [HEADER, os.path.join(ROOT, "include", "efes_testing.h")]


def declared_functions(headers=HEADERS):
    names = set()
    for h in headers:
        src = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        names |= set(re.findall(r"\b(efes_\w+)\s*\(", src))
    return sorted(names)


def test_test_hooks_are_outside_the_stable_header():
    """efes_debug_fault_after is a test hook, declared in efes_testing.h only."""
    assert "efes_debug_fault_after" not in declared_functions([HEADER])
    assert declared_functions([HEADERS[1]]) == ["efes_debug_fault_after"]


def test_every_declared_symbol_is_exported(efes_lib):
    L = ctypes.CDLL(efes_lib.LIB_PATH)
    names = declared_functions()
    assert len(names) >= 40
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    # the Python binding declares a signature for every one of them
    assert sorted(efes_lib.SIGNATURES) == names


def test_nm_shows_c_linkage(efes_lib):
    out = subprocess.run(["nm", "-D", "--defined-only", efes_lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\s[TW]\s+(efes_\w+)$", out, flags=re.M))
    assert set(declared_functions()) <= exported


def test_struct_layouts_match_header(tmp_path, efes_lib):
    prog = tmp_path / "layout.c"
    prog.write_text("""
#include <stdio.h>
#include <stddef.h>
#include "efes_hash.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu\\n", sizeof(efes_sha1_state), offsetof(efes_sha1_state, x),
         offsetof(efes_sha1_state, nx), offsetof(efes_sha1_state, len), sizeof(efes_crc32_state));
  printf("%zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(efes_job), offsetof(efes_job, length), offsetof(efes_job, sha1),
         offsetof(efes_job, crc32), offsetof(efes_job, sum), offsetof(efes_job, status), offsetof(efes_job, flags),
         offsetof(efes_job, _reserved));
  return 0;
}""")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.dirname(HEADER), str(prog), "-o", str(exe)], check=True)
    a, b = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")[:2]
    S, J = efes_lib.Sha1State, efes_lib.Job
    assert a.split() == [str(v) for v in (ctypes.sizeof(S), S.x.offset, S.nx.offset, S.len.offset, 4)]
    assert b.split() == [str(v) for v in (ctypes.sizeof(J), J.length.offset, J.sha1.offset, J.crc32.offset,
                                          J.sum.offset, J.status.offset, J.flags.offset, J._reserved.offset)]
    assert efes_lib.JOB_DTYPE.itemsize == ctypes.sizeof(J)
    assert efes_lib.SHA1_STATE_DTYPE.fields["nx"][1] == S.nx.offset


def test_host_codecs_match_golden(efes_lib, golden):
    L = efes_lib.lib()
    for case in golden["sha1_states"]:
        for text in case["texts"]:
            st = efes_lib.Sha1State()
            assert L.efes_sha1_state_unmarshal_text(ctypes.byref(st), text.encode(), 200) == 0
            out = ctypes.create_string_buffer(200)
            L.efes_sha1_state_marshal_text(ctypes.byref(st), out)
            assert out.raw.decode() == text
    st = efes_lib.Sha1State()
    assert L.efes_sha1_state_unmarshal_text(ctypes.byref(st), b"00" * 99, 198) == efes_lib.EFES_ERR_INVALID_DIGEST
    assert L.efes_sha1_state_unmarshal_text(ctypes.byref(st), b"0g" * 100, 200) == efes_lib.EFES_ERR_INVALID_DIGEST
    c = efes_lib.Crc32State()
    assert L.efes_crc32_state_unmarshal_text(ctypes.byref(c), b"0d4a1185", 8) == 0 and c.crc == 0x0D4A1185
    out = ctypes.create_string_buffer(8)
    L.efes_crc32_state_marshal_text(ctypes.byref(c), out)
    assert out.raw == b"0d4a1185"
    assert L.efes_crc32_state_unmarshal_text(ctypes.byref(c), b"0d4a118", 7) == efes_lib.EFES_ERR_INVALID_DIGEST


def test_state_init_is_newsha1(efes_lib):
    st = efes_lib.Sha1State()
    st.nx, st.len = 5, 9
    efes_lib.lib().efes_sha1_state_init(ctypes.byref(st))
    assert list(st.h) == [0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476, 0xC3D2E1F0] and st.nx == 0 and st.len == 0


def _advance_raw(t0, s, nbytes):
    for _ in range(nbytes):
        s = int(t0[s & 0xFF]) ^ (s >> 8)
    return s


def test_crc_tables(efes_lib, oracle):
    n = 8 * 256 + 7 * 4 * 256
    buf = np.zeros(n, dtype=np.uint32)
    assert efes_lib.lib().efes_crc32_tables(buf.ctypes.data, n) == n
    slice8 = buf[:2048].reshape(8, 256)
    for k in range(8):
        assert (slice8[k] == oracle.crc32_table(k)).all()
    shift = buf[2048:].reshape(7, 4, 256)
    t0 = slice8[0]
    rng = np.random.default_rng(0)
    for k in range(7):
        for v in [1, 0x80000000, int(rng.integers(0, 2**32))]:
            got = 0
            for b in range(4):
                got ^= int(shift[k, b, (v >> (8 * b)) & 0xFF])
            assert got == _advance_raw(t0, v, 64 << k), (k, hex(v))
    assert efes_lib.lib().efes_crc32_tables(buf.ctypes.data, n - 1) == efes_lib.EFES_ERR_ARG


def test_position_table_block_update(efes_lib):
    """The WIDE / grouped kernels' block CRC (efes_kernels.hip crc_issue / crc_block_pos): the raw
    register after a 64-byte block is the XOR of pos[o][byte_o] over its 64 bytes, with bytes 0..3
    XOR-ed with the old register first -- equal to crc32.go's byte-wise update (:125) and to zlib."""
    n = 8 * 256 + 7 * 4 * 256
    buf = np.zeros(n + 64 * 256, dtype=np.uint32)
    assert efes_lib.lib().efes_crc32_tables(buf.ctypes.data, buf.size) == buf.size
    t0, pos = buf[:256], buf[n:].reshape(64, 256)
    assert (pos[63] == t0).all()  # a byte with nothing after it: IEEETable
    rng = np.random.default_rng(5)
    crc = 0  # Go's crc of "" (crc32.go:68); raw register = ~crc
    data = b""
    for _ in range(24):
        block = rng.integers(0, 256, 64, dtype=np.uint8).tobytes()
        reg = (~crc) & 0xFFFFFFFF
        got = 0
        for o, b in enumerate(block):
            got ^= int(pos[o][b ^ ((reg >> (8 * o)) & 0xFF if o < 4 else 0)])
        assert got == _advance_raw_bytes(t0, reg, block)
        crc = (~got) & 0xFFFFFFFF
        data += block
        assert crc == zlib.crc32(data)


def _advance_raw_bytes(t0, s, data):
    for b in data:
        s = int(t0[(s ^ b) & 0xFF]) ^ (s >> 8)
    return s


def test_no_gpu_is_an_error_not_a_fallback(efes_lib):
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    h = ctypes.c_void_p()
    rc = efes_lib.lib().efes_ctx_create(0, ctypes.byref(h))
    assert rc == efes_lib.EFES_ERR_NO_DEVICE and not h.value
    assert efes_lib.lib().efes_strerror(rc) == b"no usable gfx950 device"


def test_crc32_combine_matches_concatenation(efes_lib):
    """efes_crc32_combine == zlib crc32 of the concatenation (crc32.go linearity)."""
    import random
    import zlib
    L = efes_lib.lib()
    rng = random.Random(4)
    for la, lb in [(0, 0), (0, 5), (5, 0), (1, 1), (63, 65), (4096, 1 << 20), (rng.randint(0, 99999), 12345)]:
        a, b = rng.randbytes(la), rng.randbytes(lb)
        assert L.efes_crc32_combine(zlib.crc32(a), zlib.crc32(b), lb) == zlib.crc32(a + b)
    # associativity over huge lengths (no data needed): ((a+b)+c) == (a+(b+c))
    ca, cb, cc = 0x12345678, 0x9ABCDEF0, 0x0F1E2D3C
    lb, lc = (1 << 40) + 3, (10 << 40) + 77
    left = L.efes_crc32_combine(L.efes_crc32_combine(ca, cb, lb), cc, lc)
    right = L.efes_crc32_combine(ca, L.efes_crc32_combine(cb, cc, lc), lb + lc)
    assert left == right


def test_integration_doc_binds_only_declared_symbols():
    """The cgo binding (go/*.go) and INTEGRATION.md only call entry points include/efes_hash.h declares."""
    for text in [open(os.path.join(ROOT, "INTEGRATION.md")).read(), "\n".join(_go_sources().values())]:
        used = set(re.findall(r"\bC\.(efes_\w+)\s*\(", text))
        missing = sorted(used - set(declared_functions()))
        assert not missing, missing
        for const in set(re.findall(r"\bC\.(EFES_\w+)", text)):
            assert re.search(r"#define\s+%s\b" % const, open(HEADER).read()), const
    assert len(set(re.findall(r"\bC\.(efes_\w+)\s*\(", "\n".join(_go_sources().values())))) >= 30


def test_plan_struct_layout_matches_header(tmp_path, efes_lib):
    """efes_plan / efes_plan_part (the batch planner's C structs) == the ctypes mirror."""
    prog = tmp_path / "plan.c"
    prog.write_text("""
#include <stdio.h>
#include <stddef.h>
#include "efes_hash.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %d\\n", sizeof(efes_plan_part), offsetof(efes_plan_part, exclusive),
         sizeof(efes_plan), offsetof(efes_plan, nparts), offsetof(efes_plan, part), offsetof(efes_plan, est_seconds),
         EFES_PLAN_MAX_PARTS);
  return 0;
}""")
    exe = tmp_path / "plan"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.dirname(HEADER), str(prog), "-o", str(exe)], check=True)
    got = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()
    P, Q = efes_lib.Plan, efes_lib.PlanPart
    assert got == [str(v) for v in (ctypes.sizeof(Q), Q.exclusive.offset, ctypes.sizeof(P), P.nparts.offset,
                                    P.part.offset, P.est_seconds.offset, efes_lib.PLAN_MAX_PARTS)]


def test_auto_mode_by_job_count(efes_lib):
    """efes_auto_mode (ctx NULL = one MI355X, 1024 SIMDs): DEEP, FED4, FED4E, GROUP4, then WIDE."""
    L = efes_lib.lib()
    G = efes_lib.MODE_GROUP
    F, FE = efes_lib.MODE_FED4, efes_lib.MODE_FED4E
    want = {1: efes_lib.MODE_DEEP, 1024: efes_lib.MODE_DEEP, 1025: F, 2048: F, 4096: F, 8192: F, 8193: FE,
            12288: FE, 12289: G[4], 16384: G[4], 16385: efes_lib.MODE_WIDE, 131072: efes_lib.MODE_WIDE}
    assert {n: L.efes_auto_mode(None, n) for n in want} == want


def test_integration_doc_covers_every_declared_symbol():
    """Every entry point of include/efes_hash.h appears in INTEGRATION.md's tables or the cgo binding
    it ships (go/*.go)."""
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read() + "\n".join(_go_sources().values())
    missing = [n for n in declared_functions() if not re.search(r"\b%s\b" % n, doc)]
    assert not missing, missing


def test_pool_close_waits_for_its_digests(efes_lib):
    """Pool.close() while digests made on the pool are alive must not free the C pool
    under them (their next Write re-reads its contexts).  The destroy is deferred to the last
    digest's free.  Host-only: a pooled digest touches no device until its first Write, so stand-in
    context handles suffice."""
    from efes_amd import hashing

    class FakeCtx:
        handle = ctypes.c_void_p(0x1000)

    pool = hashing.Pool([FakeCtx()])
    s, c = hashing.Sha1Digest(pool=pool), hashing.CRC32Digest(pool=pool)
    pool.close()
    assert pool.handle  # two digests still alive
    del s
    assert pool.handle
    del c
    assert pool.handle is None  # the last one freed it
    with pytest.raises(hashing.EfesError):
        hashing.Sha1Digest(pool=pool)


def test_pair_stats_layout(tmp_path, efes_lib):
    """efes_pair_stats (ABI 6) as the C compiler lays it out = the ctypes mirror; counters readable
    without a GPU."""
    src = tmp_path / "p.c"
    src.write_text('#include <stddef.h>\n#include <stdio.h>\n#include "efes_hash.h"\nint main(void){printf("%zu %zu %zu\\n",'
                   ' sizeof(efes_pair_stats), offsetof(efes_pair_stats, fused_bytes), offsetof(efes_pair_stats, settles));'
                   'return 0;}\n')
    exe = tmp_path / "p"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()
    P = efes_lib.PairStats
    assert [int(x) for x in out] == [ctypes.sizeof(P), P.fused_bytes.offset, P.settles.offset]
    st = P()
    assert efes_lib.lib().efes_pair_stats_get(ctypes.byref(st)) == 0


def test_integration_doc_two_build_targets():
    """the -tags efesgpu build swaps the digests for the whole binary, so the
    integration names two targets -- the storage server with the GPU digests, the single-stream CLI
    (efes write / efes drain) on the reference's unchanged pure-Go build -- with the Makefile and
    goreleaser lines, and no run-time routing between the paths."""
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = doc[doc.index("## 1. Build"):doc.index("## 2.")]
    # the server target: tagged cgo build, its own binary and archive carrying the library
    assert "CGO_ENABLED=1 go build -tags efesgpu -o $(NAME)-server" in sec
    assert "binary: efes-server" in sec and "flags: [-tags=efesgpu]" in sec
    assert "efes_amd/lib/libefeshash.so" in sec
    # the CLI target: the reference's own lines, unchanged
    assert "GOOS=linux GOARCH=amd64 CGO_ENABLED=0 go build -o $(NAME)" in sec
    assert "`Makefile:6`" in sec and "`.goreleaser.yml:9`" in sec
    for role in ("`write`", "`drain`", "`server`"):
        assert role in sec, role
    # the reason, measured: one stream on the GPU vs one core
    assert "0.085 GiB/s" in sec and "0.53–0.60 GiB/s" in sec
    assert "No binary routes between the two" in sec
    # the reference lines cited are the ones that build with CGO_ENABLED=0
    ref = "/root/reference"
    if os.path.isdir(ref):
        assert "CGO_ENABLED=0 go build" in open(os.path.join(ref, "Makefile")).read().split("\n")[5]
        assert "CGO_ENABLED=0" in open(os.path.join(ref, ".goreleaser.yml")).read().split("\n")[8]


# ---- the Go binding, go/*.go (no Go toolchain here: its ownership rules, checked as text) -----------
REF = "/root/reference"
DIGEST_FILES = ("sha1.go", "sha1_efes.go", "crc32.go", "crc32_efes.go")  # replaced under -tags efesgpu
GO_DIR = os.path.join(ROOT, "go")


def _go_sources() -> dict:
    """{file name: source} of the binding files a maintainer drops into the reference (go/*.go)."""
    return {f: open(os.path.join(GO_DIR, f)).read() for f in sorted(os.listdir(GO_DIR)) if f.endswith(".go")}


def _binding() -> str:
    return _go_sources()["hash_gpu.go"]


def _go_blocks():
    """Every piece of Go the integration ships: the go/*.go files and any Go left in INTEGRATION.md."""
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    return list(_go_sources().values()) + re.findall(r"```go\n(.*?)```", doc, flags=re.S)


def _go_funcs(src: str):
    """(receiver, type, name, body) of every top-level func of a Go source text."""
    out = []
    for m in re.finditer(r"^func (?:\((?:(\w+) )?\*?(\w+)\) )?(\w+)\(", src, flags=re.M):
        i = src.index("{", m.end())
        depth, j = 0, i
        while True:
            depth += {"{": 1, "}": -1}.get(src[j], 0)
            if depth == 0:
                break
            j += 1
        out.append((m.group(1), m.group(2), m.group(3), src[i:j + 1]))
    return out


def test_go_binding_never_copies_a_handle_holder():
    """`*d = *newSha1Handle(true)` copied a handle out of a temporary whose
    finalizer then freed it (a use-after-free on every resumed PATCH).  No Go block may assign
    through a dereference to a struct value (`*x = *y`, `*x = T{...}`) or copy a digest value."""
    for b in _go_blocks():
        assert not re.search(r"^\s*\*\w+\s*=", b, flags=re.M), re.search(r"^\s*\*\w+\s*=.*$", b, flags=re.M)
        assert not re.search(r"=\s*\*(?:d|w|\w+Handle\(|New\w+\()", b), "a dereferenced digest copied"


def test_go_binding_finalizer_is_on_the_handle_owner():
    """Every runtime.SetFinalizer target is the object whose handle field the same function
    allocates (`&x.c` / `&x.u` passed to C), so the handle lives exactly as long as its owner."""
    found = 0
    for b in _go_blocks():
        for recv, _typ, name, body in _go_funcs(b):
            for target, fin in re.findall(r"runtime\.SetFinalizer\((\w+),\s*([^)]*\)?)\)", body):
                if fin.strip() == "nil":
                    continue
                found += 1
                assert re.search(rf"&{target}\.(c|u)\b", body), (name, target)
                assert target == recv or re.search(rf"\b{target} := new\(\w+\)", body), (name, target)
    assert found >= 3  # sha1digest, crc32digest, uploadWriter


def test_go_binding_keeps_the_owner_alive_across_c_calls():
    """Every method that hands its handle (`d.c` through handle(), `w.u`) to C calls
    runtime.KeepAlive on the receiver after its last such call, so the finalizer cannot free the
    handle while C uses it.  The finalizer itself (free) and the allocation (`&d.c`, before any
    finalizer exists) are exempt."""
    checked = 0
    for b in _go_blocks():
        for recv, typ, name, body in _go_funcs(b):
            if not recv or name == "free":
                continue
            uses = [m.end() for m in re.finditer(rf"C\.efes_\w+\([^;\n]*(?<!&)\b{recv}\.(?:c|u|handle\(\))", body)]
            if not uses:
                continue
            checked += 1
            keep = [m.start() for m in re.finditer(rf"runtime\.KeepAlive\({recv}\)", body)]
            assert keep and max(keep) > max(uses), f"{typ}.{name}: no runtime.KeepAlive({recv}) after its C call"
    assert checked >= 15


def test_go_binding_replaces_the_digest_files_whole():
    """The -tags efesgpu file stands in for sha1.go, sha1_efes.go, crc32.go and crc32_efes.go (the
    _efes.go files read Go struct fields and define MarshalText/UnmarshalText, so they cannot
    compile beside it): every method the four define on sha1digest / crc32digest is defined by the
    binding, no other reference file defines one, and every package-level name of the four that
    another reference file uses is defined by the binding.  Needs the reference (skipped without)."""
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    for f in DIGEST_FILES:
        assert f"`{f}`" in doc[doc.index("## 1. Build"):doc.index("## 3.")], f
    if not os.path.isdir(REF):
        pytest.skip("reference not present")
    binding = "\n".join(_go_sources().values())
    mine = {(t, n) for r, t, n, _ in _go_funcs(binding) if r}
    mine_top = {n for r, _t, n, _ in _go_funcs(binding) if not r} | set(re.findall(r"^var (\w+)", binding, flags=re.M)) \
        | set(re.findall(r"^type (\w+)", binding, flags=re.M))
    theirs, defined = set(), set()
    for f in DIGEST_FILES:
        src = open(os.path.join(REF, f)).read()
        theirs |= {(t, n) for r, t, n, _ in _go_funcs(src) if r}
        defined |= {n for r, _t, n, _ in _go_funcs(src) if not r}
        defined |= set(re.findall(r"^(?:var|const|type) (\w+)", src, flags=re.M))
        for blk in re.findall(r"^(?:var|const) \((.*?)^\)", src, flags=re.M | re.S):
            defined |= set(re.findall(r"^\s+(\w+)", blk, flags=re.M))
    # the exported method sets (hash.Hash, encoding.TextMarshaler/TextUnmarshaler, Sum32); sha1.go's
    # unexported checkSum is its own Sum's helper and no other file calls a digest's unexported method
    assert {m for m in theirs if m[0] in ("sha1digest", "crc32digest") and m[1][0].isupper()} <= mine
    for f in sorted(os.listdir(REF)):
        if not f.endswith(".go") or f in DIGEST_FILES:
            continue
        src = open(os.path.join(REF, f)).read()
        src = re.sub(r'//.*$|"(?:\\.|[^"\\])*"|`[^`]*`', "", src, flags=re.M)  # code only
        others = {(t, n) for r, t, n, _ in _go_funcs(src) if r and t in ("sha1digest", "crc32digest")}
        assert not others, (f, others)
        used = {n for n in defined if re.search(rf"(?<![.\w]){n}\b", src)}
        assert used <= mine_top, (f, used - mine_top)


def test_library_env_vars_are_the_documented_four():
    """the product library reads exactly the sizing variables of INTEGRATION.md
    §3's table, and no source under efes_amd/csrc has an A/B build switch left."""
    names = set()
    for f in os.listdir(os.path.join(ROOT, "efes_amd", "csrc")):
        src = open(os.path.join(ROOT, "efes_amd", "csrc", f)).read()
        names |= set(re.findall(r'getenv\("(\w+)"\)', src))
        defines = set(re.findall(r"^#\s*if(?:n?def)?\s+(\w+)", src, flags=re.M)) - {"EFES_CHECKED", "EFES_BUILD_ID"}
        assert not {d for d in defines if d.startswith("EFES_")}, (f, defines)
    want = {"EFES_DIGEST_STAGING_MIB", "EFES_DIGEST_CHUNK_KIB", "EFES_DIGEST_SLOTS", "EFES_DIGEST_EVICT_MS"}
    assert names == want, names
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    for n in want:
        assert f"| `{n}` |" in doc, n


def test_integration_load_rule_and_gauges():
    """INTEGRATION.md §1 states the in-flight load below which the GPU server build
    hashes slower than the pure-Go build, from bench.py's patch_latency leg, and the gauges it names are
    the ones the binding's collector registers; the collector never opens the GPUs itself."""
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    rule = doc[doc.index("**Load rule for `efes-server`.**"):doc.index("## 2.")]
    assert "patch_latency" in rule and "8 × C uploads are in flight" in rule
    binding = _binding()
    registered = set(re.findall(r'prometheus\.NewDesc\("(efes_gpu_\w+)"', binding))
    named = set(re.findall(r"`(efes_gpu_\w+)(?:\{gpu\})?`", rule))
    assert named and named <= registered, (named, registered)
    assert "prometheus.MustRegister(gpuCollector{})" in binding
    collect = next(body for r, t, n, body in _go_funcs(binding) if n == "Collect")
    assert "pool()" not in collect and "gpuReady.Load()" in collect


def test_go_files_are_the_tagged_drop_in():
    """the cgo shim ships as files.  Every go/*.go file is `package main` under the
    `efesgpu` build constraint (its first line, then a blank line, as `go build` requires), and
    INTEGRATION.md points at the files instead of embedding the binding."""
    srcs = _go_sources()
    assert {"hash_gpu.go", "upload_gpu.go"} <= set(srcs)
    for name, src in srcs.items():
        assert src.startswith("//go:build efesgpu\n\n"), name
        assert re.search(r"^package main$", src, flags=re.M), name
        assert 'import "C"' in src, name
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    assert "go/hash_gpu.go" in doc and "go/efesgpu_build_tags.patch" in doc and "go/upload_gpu.go" in doc
    # the code lives in the files, not in the document: no fenced Go in it defines a digest method
    assert not [b for b in re.findall(r"```go\n(.*?)```", doc, flags=re.S) if re.search(r"^func |^package ", b, flags=re.M)]
    defined = {n for src in srcs.values() for r, _t, n, _ in _go_funcs(src) if r is None}
    assert len(defined) == len([n for src in srcs.values() for r, _t, n, _ in _go_funcs(src) if r is None])


def test_build_tag_patch_applies_to_the_reference(tmp_path):
    """go/efesgpu_build_tags.patch puts `//go:build !efesgpu` and a blank line above line 1 of exactly the
    four digest files (sha1.go:1, sha1_efes.go:1, crc32.go:1, crc32_efes.go:1) and nothing else;
    `patch --dry-run`, then the real apply, on a copy of the four reference files."""
    import shutil

    pt = os.path.join(GO_DIR, "efesgpu_build_tags.patch")
    text = open(pt).read()
    files = re.findall(r"^\+\+\+ b/(\S+)$", text, flags=re.M)
    assert sorted(files) == sorted(DIGEST_FILES)
    added = re.findall(r"^\+(?!\+\+ )(.*)$", text, flags=re.M)
    assert added == ["//go:build !efesgpu", ""] * 4
    assert not re.findall(r"^-(?!-- )", text, flags=re.M)  # removes nothing
    if not shutil.which("patch"):
        pytest.skip("patch(1) not installed")
    if not os.path.isdir(REF):
        pytest.skip("reference not present")
    for f in DIGEST_FILES:
        shutil.copy(os.path.join(REF, f), tmp_path / f)
    r = subprocess.run(["patch", "-p1", "--dry-run", "-i", pt], cwd=tmp_path, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    r = subprocess.run(["patch", "-p1", "-i", pt], cwd=tmp_path, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    for f in DIGEST_FILES:
        got = (tmp_path / f).read_text()
        assert got == "//go:build !efesgpu\n\n" + open(os.path.join(REF, f)).read(), f


def test_go_pool_opens_every_device_and_skips_failures():
    """pool() loops to efes_device_count(), and a device whose context fails
    (EFES_ERR_NO_DEVICE / _HIP / _NOMEM on a GPU that exists) is logged, counted and SKIPPED --
    `continue`, never `break` -- so one bad GPU 3 does not leave GPUs 4-7 unused; the collector
    publishes efes_gpu_devices_visible / efes_gpu_devices_opened and labels per-GPU series by HIP
    ordinal.  (The same loop runs on a GPU in tests/c/efes_consumer_test.c `enumerate`.)"""
    b = _binding()
    body = next(body for r, t, n, body in _go_funcs(b) if n == "pool")
    assert "C.efes_device_count()" in body
    loop = body[body.index("for dev := 0; dev < gpuVisible; dev++"):]
    fail = loop[loop.index("!= C.EFES_OK {"):]
    fail = fail[:fail.index("}")]
    assert "continue" in fail and "break" not in loop.split("gpuCtxs = append")[0]
    assert "gpuSkipped = append" in fail and "gpuLog.Warningln" in fail
    assert "gpuDevs = append(gpuDevs, dev)" in loop
    registered = set(re.findall(r'prometheus\.NewDesc\("(efes_gpu_\w+)"', b))
    assert {"efes_gpu_devices_visible", "efes_gpu_devices_opened"} <= registered
    collect = next(body for r, t, n, body in _go_funcs(b) if n == "Collect")
    assert "len(gpuCtxs)" in collect and "gpuVisible" in collect and "strconv.Itoa(gpuDevs[i])" in collect


def test_library_is_built_from_these_sources(efes_lib):
    """efes_build_id() of the in-tree library == efes_amd.build.source_id() of the sources beside it
    (a stale .so fails here, and the same check runs on the GPU box: tests/test_gpu_parity.py)."""
    from efes_amd import build

    assert efes_lib.lib().efes_build_id().decode() == build.source_id()


def _go_code(src: str) -> str:
    """src without comments and string literals (Go's lexical rules, enough for these files)."""
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    src = re.sub(r'"(?:\\.|[^"\\\n])*"|`[^`]*`', '""', src)
    return re.sub(r"//[^\n]*", "", src)


def test_go_files_import_exactly_what_they_use():
    """No Go compiler here, so the compile errors that are cheap to see are checked as text: Go rejects
    an unused import and a use of a package that is not imported, and every brace and parenthesis must
    balance (go/*.go)."""
    for name, src in _go_sources().items():
        imports = re.search(r'^import \((.*?)^\)', src, flags=re.M | re.S).group(1)
        pkgs = {}
        for line in imports.splitlines():
            m = re.match(r'\s*(\w+\s+)?"([\w./-]+)"', line)
            if m:
                pkgs[(m.group(1) or "").strip() or m.group(2).rsplit("/", 1)[-1]] = m.group(2)
        code = _go_code(src.split(imports, 1)[1])
        for alias in pkgs:
            assert re.search(rf"(?<![\w.]){alias}\.", code), (name, "unused import", pkgs[alias])
        std_used = set(re.findall(r"(?<![\w.])(errors|fmt|io|os|runtime|strconv|sync|atomic|unsafe|log|prometheus)\.\w", code))
        assert std_used <= set(pkgs), (name, "not imported", std_used - set(pkgs))
        whole = _go_code(src)
        for a, b in ("{}", "()", "[]"):
            assert whole.count(a) == whole.count(b), (name, a + b)


def test_go_files_use_only_declared_c_types_and_fields():
    """Every C type the cgo files name (`C.efes_*`, `C.uint32_t`, ...) is declared by include/efes_hash.h or
    is a standard C type, and every field they read from a C struct (`st.free_uploads`, `ps.settles`, ...)
    is a member of that struct in the header -- compile errors cgo would report, checked as text."""
    hdr = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    types = set(re.findall(r"typedef struct (\w+)", hdr)) | set(re.findall(r"}\s*(\w+);", hdr))
    members = {}
    for name, body in re.findall(r"typedef struct (\w+) \{(.*?)\}", hdr, flags=re.S):
        members[name] = set(re.findall(r"(\w+)(?:\[\w*\])?;", body))
    std = {"int", "char", "size_t", "uint8_t", "uint32_t", "uint64_t", "int32_t", "int64_t",
           "GoString", "CString", "GoBytes"}  # cgo's own helpers
    funcs = set(declared_functions())
    for name, src in _go_sources().items():
        code = _go_code(src)
        used = set(re.findall(r"\bC\.(\w+)", code))
        consts = {u for u in used if u.isupper() or u.startswith("EFES_")}
        unknown = used - funcs - types - std - consts
        assert not unknown, (name, unknown)
        # fields read from stats structs: `var st C.efes_queue_stats` ... `st.field`
        for var, ctype in re.findall(r"var (\w+) C\.(\w+)", code):
            if ctype in members:
                for field in set(re.findall(rf"\b{var}\.(\w+)", code)):
                    assert field in members[ctype], (name, ctype, field)
