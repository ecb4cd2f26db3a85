"""Rank-count-aware tier defaults and the topology-keyed tune store (VERDICT r5 Next #4;
mp4x/parallel/tiers.py).  CPU: the model is pure arithmetic; the store round trip runs real
device engines on gloo (CPU tensors) in successive jobs."""
import json
import math
import os

import pytest

torch = pytest.importorskip("torch")

from harness import run_ranks  # noqa: E402
from mp4x import Operators  # noqa: E402
from mp4x.parallel import tiers  # noqa: E402

SLOT = 4 << 20


def test_crossover_follows_the_per_link_model():
    b, L = 2.5, 64.0
    assert math.isinf(tiers.oneshot_crossover(2, b, L))         # same bytes, one barrier fewer
    for p in (3, 4, 8):
        s = tiers.oneshot_crossover(p, b, L)
        t1, t2 = tiers.model_times_us(p, int(s), b, L)
        assert abs(t1 - t2) < 1e-6 * t1                          # the two schedules tie at S*
        lo1, lo2 = tiers.model_times_us(p, int(s) // 2, b, L)
        hi1, hi2 = tiers.model_times_us(p, int(s) * 2, b, L)
        assert lo1 < lo2 and hi1 > hi2                           # one-shot below, two-shot above
    # the crossover falls as p grows: the two-shot's per-link share 2S/p shrinks
    assert tiers.oneshot_crossover(3, b, L) > tiers.oneshot_crossover(4, b, L) > tiers.oneshot_crossover(8, b, L)


def test_default_oneshot_limits_per_rank_count():
    got = {p: tiers.oneshot_max(p, SLOT, 2.5, 64.0) for p in (2, 3, 4, 5, 6, 7, 8)}
    assert got == {2: SLOT, 3: 512 << 10, 4: 256 << 10, 5: 256 << 10, 6: 256 << 10, 7: 256 << 10, 8: 256 << 10}
    # a slower barrier moves the crossover up, a faster link too; always within [64 KiB, slot]
    assert tiers.oneshot_max(8, SLOT, 10.0, 64.0) == 1 << 20
    assert tiers.oneshot_max(8, SLOT, 0.1, 10.0) == tiers.MIN_ONESHOT
    assert tiers.oneshot_max(4, SLOT, 100.0, 100.0) == SLOT


def test_engine_uses_the_model(monkeypatch):
    """The staged allreduce's one-shot limit at p = 2 / 3 / 4 / 8 is the model's (the latency
    tier's 256 KiB stays the floor); MP4X_IPC_ONESHOT_MAX overrides it."""
    from mp4x.parallel.device_engine import DeviceEngine
    from mp4x.parallel.coll import LoopbackHub

    monkeypatch.delenv("MP4X_IPC_ONESHOT_MAX", raising=False)
    for p, want in ((2, SLOT), (3, 512 << 10), (4, 256 << 10), (8, 256 << 10)):
        from mp4x.parallel.coll import _FakeComm
        e = DeviceEngine(_FakeComm(0, p), coll=LoopbackHub(p).coll(0), device="cpu")
        assert e._oneshot_limit() == want, (p, e._oneshot_limit())
    monkeypatch.setenv("MP4X_IPC_ONESHOT_MAX", str(128 << 10))
    e = DeviceEngine(_FakeComm(0, 2), coll=LoopbackHub(2).coll(0), device="cpu")
    assert e._oneshot_limit() == 128 << 10


def test_topology_key_is_stable_and_distinguishes():
    a = {"p": 8, "device": "AMD Instinct MI355X", "backend": "nccl", "xgmi": {"pairs": {"xgmi": 56}}}
    b = dict(a, p=4)
    c = dict(a, xgmi={"pairs": {"pcie": 56}})
    assert tiers.topology_key(a) == tiers.topology_key(json.loads(json.dumps(a)))
    assert len({tiers.topology_key(x) for x in (a, b, c)}) == 3
    assert tiers.tune_path(a) != tiers.tune_path(c)


def _tune_job(comm, mode):
    eng = comm.device
    loaded = dict(eng._tuned)
    if mode == "write":
        t = torch.ones(4096, dtype=torch.float32)
        eng.autotune_allreduce(t, Operators.Float.SUM, iters=1)
        comm.peer_barrier()
    return {"loaded": {str(k): v for k, v in loaded.items()}, "tuned": {str(k): v for k, v in eng._tuned.items()},
            "path": eng.tune_path()}


def test_tune_store_is_loaded_by_the_next_job_with_the_same_key(tmp_path):
    env = {"MP4X_TUNE_AUTO": "1", "MP4X_TUNE_DIR": str(tmp_path), "MP4X_AUTOTUNE_EXTRA": "1"}
    res, code, _ = run_ranks(2, _tune_job, args=("write",), timeout=120, env=env)
    assert code == 0
    path = res[0]["path"]
    assert path.startswith(str(tmp_path)) and os.path.exists(path)
    written = res[0]["tuned"]
    assert written and all(not r["loaded"] for r in res.values())
    # the next job on the same topology pins the table at creation, on every rank
    res2, code, _ = run_ranks(2, _tune_job, args=("read",), timeout=120, env=env)
    assert code == 0 and all(r["loaded"] == written for r in res2.values()), res2
    # another topology key (3 ranks) never reads it
    res3, code, _ = run_ranks(3, _tune_job, args=("read",), timeout=120, env=env)
    assert code == 0 and all(not r["loaded"] for r in res3.values())
    assert res3[0]["path"] != path
    # a file under the right name whose recorded topology differs is refused (nothing pinned)
    with open(path) as f:
        table = json.load(f)
    table["topology"] = dict(table["topology"], device="other")
    with open(path, "w") as f:
        json.dump(table, f)
    res4, code, _ = run_ranks(2, _tune_job, args=("read",), timeout=120, env=env)
    assert code == 0 and all(not r["loaded"] for r in res4.values())
    # without MP4X_TUNE_AUTO nothing is read or written
    env_off = dict(env, MP4X_TUNE_AUTO="0")
    res5, code, _ = run_ranks(2, _tune_job, args=("read",), timeout=120, env=env_off)
    assert code == 0 and all(not r["loaded"] and r["path"] is None for r in res5.values())


def test_pins_between_measured_classes_follow_the_measurement():
    """A size class the tier sweep did not visit takes the schedule its two measured neighbours
    (same kind, dtype, op) both pinned; neighbours that disagree leave it to the tier defaults."""
    from mp4x.parallel.autotune import _TunedTable
    t = _TunedTable()
    f32, f64 = torch.float32, torch.float64
    t[(f32, 0, 12)] = "ipc1"           # 4 KiB
    t[(f32, 0, 16)] = "ipc1"           # 64 KiB
    t[(f32, 0, 18)] = "ipc2"           # 256 KiB
    t[("reduce", f32, 0, 20)] = "rccl"
    t[("reduce", f32, 0, 24)] = "rccl"
    assert t.pinned((f32, 0, 14)) == "ipc1"          # between two ipc1 pins
    assert t.pinned((f32, 0, 17)) is None            # ipc1 below, ipc2 above: the defaults decide
    assert t.pinned((f32, 0, 18)) == "ipc2"          # an exact pin
    assert t.pinned((f32, 0, 10)) is None            # below every measurement
    assert t.pinned((f32, 0, 30)) is None            # above every measurement
    assert t.pinned((f64, 0, 14)) is None            # another dtype
    assert t.pinned((f32, 1, 14)) is None            # another op
    assert t.pinned(("reduce", f32, 0, 22)) == "rccl"
    assert t.pinned(("broadcast", f32, 0, 22)) is None
