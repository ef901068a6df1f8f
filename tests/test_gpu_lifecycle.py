"""The Go binding's object lifecycle under AddressSanitizer (tests/c/efes_lifecycle_test.c
built by tools/asan_build.sh with the library's host code instrumented): json's resume sequence of
fileinfo.go:43 -- a zero digest, UnmarshalText opening its handle in place -- beside a collector thread
freeing every earlier PATCH's digests, from 8 request threads, every text and digest equal to the
oracle's, and no sanitizer report.  The negative control replays round 4's `*d = *newSha1Handle(true)`
and must die with heap-use-after-free: the test sees the bug class it guards against."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "c", "efes_lifecycle_test_asan")
# LeakSanitizer off: the HIP runtime keeps allocations until exit by design
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1")


@pytest.fixture(scope="module")
def exe():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if not os.path.exists(EXE):
        pytest.fail(f"{EXE} not built (__graft_entry__.build() runs tools/asan_build.sh)")
    return EXE


def test_binding_lifecycle_is_clean_under_asan(exe):
    r = subprocess.run([exe, "fixed", "8", "3"], capture_output=True, text=True, timeout=110, env=ENV)
    assert "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0 and "efes_lifecycle_test ok" in r.stdout, (r.stdout, r.stderr[-4000:])


def test_round4_binding_is_caught_as_use_after_free(exe):
    r = subprocess.run([exe, "old"], capture_output=True, text=True, timeout=110, env=ENV)
    assert r.returncode != 0, (r.stdout, r.stderr[-4000:])
    assert "heap-use-after-free" in r.stderr, r.stderr[-4000:]
