"""Host logic of efes_plan_batch (no GPU: planning is host-only, ctx = NULL assumes one MI355X).

The planner orders a batch longest-first and splits it between a DEEP / grouped-DEEP launch
(the long jobs) and a WIDE launch (the rest) by an issue-time model (efes_plan.cpp)."""
import numpy as np
import pytest

from efes_amd._lib import MODE_DEEP, MODE_FED4, MODE_FED4E, MODE_GROUP, MODE_WIDE
from efes_amd.hashing import plan_batch

MiB = 1 << 20


def test_order_is_stable_longest_first():
    rng = np.random.default_rng(1)
    lengths = rng.integers(0, 5, 1000).astype(np.uint64) * 4096
    order, plan = plan_batch(lengths)
    assert sorted(order.tolist()) == list(range(1000))
    got = lengths[order]
    assert (np.diff(got.astype(np.int64)) <= 0).all()
    for v in np.unique(lengths):  # stable within equal lengths
        idx = order[got == v]
        assert (np.diff(idx.astype(np.int64)) > 0).all()
    assert plan.njobs == 1000 and sum(p[0] for p in plan.parts()) == 1000


def test_metric_config_goes_deep():
    """BASELINE configs[1]/[2]: 1024 x 4 MiB = one job per SIMD -> all DEEP (one wave per job)."""
    _, plan = plan_batch([4 * MiB] * 1024)
    assert [(j, m) for j, m, _ in plan.parts()] == [(1024, MODE_DEEP)]


def test_ingest_config_goes_wide():
    """BASELINE configs[4] per launch: 131072 x 4 MiB -> throughput-bound, all WIDE."""
    _, plan = plan_batch([4 * MiB] * 131072)
    assert plan.parts() == [(131072, MODE_WIDE, False)]


def test_mixed_config_splits_longest_class_off():
    """BASELINE configs[3]: ChunkSize 64K..64M -> the longest classes in deep shapes on CUs of
    their own, the rest WIDE on the other CUs."""
    sizes = np.asarray([64 << 10 << i for i in range(11)], dtype=np.uint64)
    lengths = sizes[np.random.default_rng(7).integers(0, 11, 65536)]
    order, plan = plan_batch(lengths)
    parts = plan.parts()
    assert len(parts) in (2, 3) and sum(p[0] for p in parts) == 65536
    for jobs, mode, exclusive in parts[:-1]:  # deep shapes (or lone-wave WIDE) on CUs of their own
        assert mode in (MODE_FED4, MODE_FED4E, MODE_WIDE, *MODE_GROUP.values()) and exclusive
    assert parts[-1][1] == MODE_WIDE and not parts[-1][2]
    # cuts fall between lengths: every job of a part is at least as long as every later one
    cut = 0
    for jobs, _, _ in parts[:-1]:
        cut += jobs
        assert lengths[order[cut - 1]] > lengths[order[cut]]
    assert lengths[order[0]] == 64 * MiB
    assert 0.5 < plan.est_seconds < 2.0


def test_more_long_jobs_than_simds_use_fed_then_groups():
    """Up to 32 long jobs per CU: FED4 (DEEP's latency); beyond that grouped DEEP."""
    _, plan = plan_batch([4 * MiB] * 4096)
    assert len(plan.parts()) == 1 and plan.parts()[0][1] == MODE_FED4
    _, plan = plan_batch([4 * MiB] * 16384)
    assert len(plan.parts()) == 1 and plan.parts()[0][1] in MODE_GROUP.values()


def test_empty_and_zero_lengths():
    order, plan = plan_batch([])
    assert plan.njobs == 0 and plan.nparts == 0 and order.size == 0
    order, plan = plan_batch([0, 0, 0])
    assert plan.njobs == 3 and sorted(order.tolist()) == [0, 1, 2] and sum(p[0] for p in plan.parts()) == 3


@pytest.mark.parametrize("force,expect", [
    ("8:100", [(100, MODE_GROUP[8], False), (2900, MODE_WIDE, False)]),
    ("64:5000", [(3000, MODE_DEEP, False)]),
    ("4:10x,16:20", [(10, MODE_GROUP[4], True), (20, MODE_GROUP[16], False), (2970, MODE_WIDE, False)]),
    ("0:3000", [(3000, MODE_WIDE, False)]),
    ("0:5x", [(5, MODE_WIDE, True), (2995, MODE_WIDE, False)]),
])
def test_caller_built_plan(force, expect):
    """efes_plan is a plain struct a caller may fill itself (efes_amd.batch.forced_plan builds one from
    a spec; the GPU tests force every part shape through efes_hash_submit_plan with it).  Round 5
    removed the library's EFES_PLAN_FORCE environment override: a deployment's environment can no
    longer change which kernels hash production bytes."""
    from efes_amd.batch import forced_plan

    plan = forced_plan(3000, force)
    assert plan.njobs == 3000 and plan.parts() == expect


def test_caller_built_plan_rejects_too_many_parts():
    from efes_amd.batch import forced_plan

    with pytest.raises(ValueError):
        forced_plan(3000, "4:10,8:10,16:10,32:10")
    with pytest.raises(ValueError):
        forced_plan(3000, "3:10")


def test_planner_ignores_the_removed_override(monkeypatch):
    """The old EFES_PLAN_FORCE variable set in the environment changes nothing."""
    _, model = plan_batch([MiB] * 3000)
    monkeypatch.setenv("EFES_PLAN_FORCE", "8:100")
    _, plan = plan_batch([MiB] * 3000)
    assert plan.parts() == model.parts()


def test_batch_larger_than_max_jobs_is_rejected():
    """EFES_MAX_JOBS (efes_hash.h): a count beyond it is EFES_ERR_ARG before anything is read."""
    import ctypes

    from efes_amd._lib import EFES_ERR_ARG as ERR_ARG, Plan, lib

    one = (ctypes.c_uint64 * 1)(64)
    order = (ctypes.c_uint32 * 1)()
    plan = Plan()
    assert lib().efes_plan_batch(None, one, (1 << 30) + 1, order, ctypes.byref(plan)) == ERR_ARG
    assert lib().efes_plan_batch(None, one, 1, order, ctypes.byref(plan)) == 0


def test_mixed_config_deep_part_runs_in_rounds():
    """configs[3] under the LPT placement model: FED4E takes the 64 MiB class on 126 CUs and the
    GROUP4 part holds several classes (32, 16, 8 MiB: more workgroups than the 130 CUs left, so
    it runs in rounds), which brings the step to the FED4E part's end (measured 0.884 s,
    profiles/r02_plan_lpt/)."""
    sizes = np.asarray([64 << 10 << i for i in range(11)], dtype=np.uint64)
    lengths = sizes[np.random.default_rng(7).integers(0, 11, 65536)]
    order, plan = plan_batch(lengths)
    parts = plan.parts()
    assert parts[0][1] == MODE_FED4E and parts[0][2]
    assert lengths[order[0]] == 64 * MiB and lengths[order[parts[0][0] - 1]] == 64 * MiB
    g4 = parts[1]
    assert g4[1] == MODE_GROUP[4] and g4[2]
    cls = set(lengths[order[parts[0][0]:parts[0][0] + g4[0]]].tolist())
    assert len(cls) >= 2 and max(cls) == 32 * MiB
    assert 0.85 < plan.est_seconds < 0.95


@pytest.mark.parametrize("seed", range(12))
def test_random_batches_give_valid_plans(seed):
    """Any batch: parts cover it exactly, cuts fall on length boundaries, deep parts are
    exclusive and precede the shared WIDE part, the estimate is positive."""
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 40000))
    kind = seed % 3
    if kind == 0:
        lengths = rng.integers(0, 1 << 26, n)
    elif kind == 1:
        lengths = np.exp(rng.uniform(np.log(1 << 12), np.log(1 << 26), n)).astype(np.int64)
    else:
        lengths = rng.choice([0, 1, 64, 4096, 1 << 20, 4 << 20, 64 << 20], n)
    lengths = lengths.astype(np.uint64)
    order, plan = plan_batch(lengths)
    parts = plan.parts()
    assert 1 <= len(parts) <= 4 and sum(p[0] for p in parts) == n
    assert sorted(order.tolist()) == list(range(n))
    cut = 0
    for i, (jobs, mode, excl) in enumerate(parts):
        assert jobs > 0
        if mode != MODE_WIDE or i < len(parts) - 1:
            assert excl or len(parts) == 1
        if i < len(parts) - 1:
            cut += jobs
            assert lengths[order[cut - 1]] >= lengths[order[cut]]
    assert plan.est_seconds > 0
