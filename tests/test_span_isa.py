"""The span kernel's M0 contract, checked in its gfx950 ISA (CPU).

`fetch_row` (efes_amd/csrc/efes_crc_span.hip:152-160) writes M0 -- the LDS address of a
`global_load_lds_dwordx4` -- from inline assembly.  LLVM treats M0 as a reserved register: listing it
as an asm clobber is not honoured (clang warns "Reserved registers on the clobber list may not be
preserved across the asm statement" and emits the same code), so nothing in the source stops a later
compiler from keeping a value of its own in M0 across these statements.  This test is the guard: it
compiles the kernel file to assembly and checks span_kernel's body --
  * every M0 write is `s_mov_b32 m0, sN`, followed by `s_nop 0` and then `global_load_lds_dwordx4`
    (one wait state between the write and the DMA that reads it);
  * nothing else in the body reads or writes M0;
  * M0 writes and LDS-DMA loads are equal in number.
The checker is shown to fail on hand-mutated copies of the same assembly."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "efes_amd", "csrc", "efes_crc_span.hip")
KERNEL = "_ZN4efes11span_kernelENS_8SpanArgsE"


def kernel_body(asm: str, name: str = KERNEL) -> list[str]:
    """The instruction lines of `name` (label to its .Lfunc_end), comments and directives dropped."""
    lines = asm.splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith(name + ":"))
    out = []
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        s = l.split(";")[0].strip()
        if s and not s.startswith(".") and not s.endswith(":"):
            out.append(s)
    return out


def m0_violations(body: list[str]) -> list[str]:
    """Every departure from the contract in the module docstring (empty: the body keeps it)."""
    bad = []
    writes = loads = 0
    for i, ins in enumerate(body):
        if "global_load_lds" in ins:
            loads += 1
        if not re.search(r"\bm0\b", ins):
            continue
        if not re.fullmatch(r"s_mov_b32 m0, s\d+", ins):
            bad.append(f"{i}: M0 used outside the LDS-DMA pattern: {ins}")
            continue
        writes += 1
        nxt = body[i + 1:i + 3]
        if len(nxt) < 2 or nxt[0] != "s_nop 0" or not nxt[1].startswith("global_load_lds_dwordx4"):
            bad.append(f"{i}: M0 write not followed by s_nop 0 + global_load_lds_dwordx4: {nxt}")
    if writes != loads:
        bad.append(f"{writes} M0 writes for {loads} LDS-DMA loads")
    if writes == 0:
        bad.append("no LDS-DMA site found (kernel renamed or restructured?)")
    return bad


@pytest.fixture(scope="module")
def span_asm(tmp_path_factory):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("span_isa") / "span.s"
    # the flags of efes_amd/build.py's product build, device code only
    subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", os.path.join(ROOT, "include"),
                    "--cuda-device-only", "-S", SRC, "-o", str(out)], check=True, capture_output=True, timeout=300)
    return out.read_text()


def test_span_kernel_m0_only_feeds_its_lds_dma(span_asm):
    body = kernel_body(span_asm)
    assert m0_violations(body) == []
    # today's kernel: the prologue fetch and the loop's next-row fetch, four 1 KiB loads each
    assert sum("global_load_lds_dwordx4" in i for i in body) == 8


def test_checker_rejects_mutated_assembly(span_asm):
    body = kernel_body(span_asm)
    w = next(i for i, ins in enumerate(body) if ins.startswith("s_mov_b32 m0,"))
    mutants = {
        "compiler keeps a value in M0": body[:3] + ["s_mov_b32 s7, m0"] + body[3:],
        "M0 as an operand elsewhere": body[:w] + ["s_add_u32 m0, m0, 4"] + body[w:],
        "missing wait state": body[:w + 1] + body[w + 2:],
        "M0 written with no DMA after it": body[:w] + ["s_mov_b32 m0, s3", "s_nop 0", "v_mov_b32_e32 v1, v2"] + body[w:],
        "DMA without its M0 write": body + ["global_load_lds_dwordx4 v[6:7], off nt"],
    }
    for what, m in mutants.items():
        assert m0_violations(m), what
