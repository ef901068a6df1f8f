"""bench.py's host-side machinery without a GPU (the round-5 r05_check stall, DESIGN_NOTES.md §5).

The clock meter's amdsmi half must never hold the bench: amdsmi is initialised once per process
(however many meters), and a poll call that blocks is abandoned after SMI_JOIN_S with a note in the
leg's `clock` instead of a join that waits for good.  A stand-in `amdsmi` module plays the part."""
import sys
import threading
import time
import types

import pytest


@pytest.fixture
def bench(monkeypatch, tmp_path):
    import bench as b
    monkeypatch.setattr(b, "ROOT", str(tmp_path))  # no tools/libclockprobe.so: the amdsmi half alone
    monkeypatch.setattr(b, "_SMI_STATE", {"module": None, "tried": False, "stuck": False})
    monkeypatch.setattr(b, "SMI_JOIN_S", 0.5)
    return b


def _fake_amdsmi(monkeypatch, block_after: int):
    fake = types.ModuleType("amdsmi")
    gate = threading.Event()
    n = {"init": 0, "calls": 0, "shut": 0}

    def init():
        n["init"] += 1

    def metrics(_h):
        n["calls"] += 1
        if n["calls"] > block_after:
            gate.wait(30)  # a driver call that does not come back
        return {"current_gfxclks": [2400, 2390]}

    fake.amdsmi_init = init
    fake.amdsmi_shut_down = lambda: n.__setitem__("shut", n["shut"] + 1)
    fake.amdsmi_get_processor_handles = lambda: ["gpu0"]
    fake.amdsmi_get_gpu_device_bdf = lambda _h: "0000:05:00.0"
    fake.amdsmi_get_gpu_metrics_info = metrics
    monkeypatch.setitem(sys.modules, "amdsmi", fake)
    return n, gate


def test_clock_meter_polls_and_inits_amdsmi_once(bench, monkeypatch):
    n, _ = _fake_amdsmi(monkeypatch, block_after=10 ** 9)
    for _ in range(3):
        m = bench.ClockMeter(0)
        m.start(0)
        time.sleep(0.1)
        m.end(0)
        out = m.stop()
        assert out["smi_samples"] > 5 and out["smi_mhz_mean"] == 2395.0 and out["mhz"] == 2395.0
    assert n["init"] == 1  # one amdsmi_init for the process, not one per meter


def test_clock_meter_abandons_a_blocking_amdsmi_call(bench, monkeypatch):
    n, gate = _fake_amdsmi(monkeypatch, block_after=3)
    m = bench.ClockMeter(0)
    m.start(0)
    time.sleep(0.1)  # the poll thread is now stuck inside the fourth metrics call
    m.end(0)
    t0 = time.perf_counter()
    out = m.stop()
    took = time.perf_counter() - t0
    try:
        assert took < 0.5 + 1.0, took  # bounded by SMI_JOIN_S, not by the stuck call
        assert "did not return" in out["smi_note"] and "smi_mhz_mean" not in out
        assert m.smi is None and bench._SMI_STATE["stuck"]  # dropped for the rest of the process
        m.start(0)  # the next region runs without amdsmi, at once
        m.end(0)
        assert m.stop().get("smi_samples") is None
    finally:
        gate.set()


def test_legs_time_and_log_each_leg(bench, capsys):
    legs = bench.Legs()
    assert legs.run("one", lambda x: x + 1, 1) == 2
    assert set(legs.seconds) == {"one"} and legs.seconds["one"] >= 0
    err = capsys.readouterr().err
    assert "[bench] one: start" in err and "[bench] one: done in" in err
