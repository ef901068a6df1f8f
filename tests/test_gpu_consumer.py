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


def test_c_consumer_enumerates_past_a_failing_device():
    """go/hash_gpu.go pool()'s loop, run by the C consumer over the ordinals
    0, <efes_device_count()>, 0 -- a middle ordinal whose efes_ctx_create fails (out of range here: a
    one-GPU box has no second card to fail; the loop treats every failing code alike) between two that
    open (two contexts of GPU 0 stand in for two GPUs).  The failure is reported and skipped, the pool
    holds both contexts, pooled resumable uploads equal the oracle, and the context opened AFTER the
    failure hashes too."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if not os.path.exists(EXE):
        pytest.fail(f"{EXE} not built (__graft_entry__.build())")
    n = torch.cuda.device_count()
    r = subprocess.run([EXE, "enumerate", f"0,{n},0", "16", "4"], capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "efes_consumer_test ok (enumerate)" in r.stdout, r.stdout
    assert f"device {n} skipped: invalid argument" in r.stdout, r.stdout
    assert f"visible {n}, listed 3, opened 2, skipped 1" in r.stdout, r.stdout
