"""The upload receiver above the C ABI (efes_amd/host/efes_receiver.hpp: the C++ mirror of
fileinfo.go, filereceiver.go and sha1file.go) driven by the reference's own tests, replayed in
tests/cpp/receiver_test.cpp with every digest and every `.info` byte checked against the oracle.

cpu: the `.info` JSON codec (json.Encoder / Decoder semantics), strconv / filepath helpers, and
     the handler paths that end before any hashing (POST, HEAD, DELETE, 400, 409).
gpu: filereceiver_test.go's six tests with the digest headers asserted (KATs for "foo", "baz",
     "foobar", ""), sha1file_test.go over a real file, write.go's sendFile (client Sha1File and
     server saveFile both on the GPU) over a connection that breaks PATCHes mid-body, 16 threads
     of resumable uploads through ServeHTTP, and saveFile's error paths (broken body, vanished
     file, Go panic states)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "cpp", "receiver_test")


def _run(args, timeout, env=None):
    if not os.path.exists(EXE):
        pytest.fail(f"{EXE} not built (__graft_entry__.build())")
    return subprocess.run([EXE] + args, capture_output=True, text=True, timeout=timeout,
                          env=dict(os.environ, **(env or {})))


def test_receiver_cpu(tmp_path):
    r = _run(["cpu", str(tmp_path)], 60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "receiver_test cpu ok" in r.stdout, r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("copybuf", ["copybuf", "reserve"], ids=["copybuf", "reserve_commit"])
def test_receiver_gpu(tmp_path, copybuf):
    """saveFile's two staging paths: io.Copy's buffer + efes_upload_write (default) and the body read
    straight into the pinned staging (efes_upload_reserve/commit, SetSaveFileCopyBuffer(false))."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    r = _run(["gpu", str(tmp_path), "16", "4", copybuf], 110)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "receiver_test gpu ok" in r.stdout, r.stdout
