"""The C ABI driven by a plain C consumer (tests/c/efes_consumer_test.c): concurrent resumable
uploads PATCH by PATCH as filereceiver.go:171-227 runs them (UnmarshalText -> 32 KiB Writes ->
MarshalText / Sum), batched device jobs in every kernel shape, and the error codes -- each
checked against the CPU oracle inside the program."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "c", "efes_consumer_test")


def test_c_consumer():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if not os.path.exists(EXE):
        pytest.fail(f"{EXE} not built (__graft_entry__.build())")
    r = subprocess.run([EXE, "16", "6"], capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "efes_consumer_test ok" in r.stdout, r.stdout
