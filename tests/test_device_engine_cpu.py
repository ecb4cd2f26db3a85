"""Device-engine algorithm logic on CPU (gloo backend, CPU tensors, world_size 2-4).

The GPU engine's schedules (RCCL collective, a2a two-shot with rank-ordered reduce, p2p
gather/scatter/allgather-v, reduce = RS + gather) are exercised here with the gloo backend so
the distributed path is covered by construction before it runs on MI355X.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from harness import run_ranks  # noqa: E402
from mp4x import CommUtils, Operands, Operators  # noqa: E402


def engine_matrix(comm, algo):
    import os
    os.environ["MP4X_DEVICE_ALGO"] = algo
    eng = comm.device
    eng.algo = algo
    p, r = comm.getSlaveNum(), comm.getRank()
    n = 1001
    # allreduce SUM (allreduce split: last rank takes the remainder)
    t = torch.full((n,), float(r + 1), dtype=torch.float64)
    eng.allreduce(t, 3, n - 2, Operators.Double.SUM)
    assert torch.all(t[3:n - 2] == p * (p + 1) / 2) and t[0] == r + 1
    # ops RCCL lacks -> always the a2a schedule + rank-ordered reduce
    x = torch.full((n,), 1 << r, dtype=torch.int32)
    eng.allreduce(x, 0, n, Operators.Int.BITS_OR)
    assert torch.all(x == (1 << p) - 1)
    s = torch.full((n,), r + 1, dtype=torch.int16)
    eng.allreduce(s, 0, n, Operators.Short.SUM)
    assert torch.all(s == p * (p + 1) // 2)
    # int16 through the data-movement collectives (RCCL / gloo have no int16: moved as bytes)
    fr, to = CommUtils.createProcessArrayFroms(n, p), CommUtils.createProcessArrayTos(n, p)
    s = torch.full((n,), -1, dtype=torch.int16)
    s[fr[r]:to[r]] = r
    eng.allgather(s, fr, to)
    assert all(torch.all(s[fr[i]:to[i]] == i) for i in range(p))
    s = torch.full((n,), -1, dtype=torch.int16)
    s[fr[r]:to[r]] = r
    eng.gather(s, fr, to, p - 1)
    assert r != p - 1 or all(torch.all(s[fr[i]:to[i]] == i) for i in range(p))
    s = torch.arange(n, dtype=torch.int16) if r == 0 else torch.zeros(n, dtype=torch.int16)
    eng.scatter(s, fr, to, 0)
    assert torch.all(s[fr[r]:to[r]] == torch.arange(fr[r], to[r], dtype=torch.int16))
    s = torch.full((n,), 3 if r == 0 else 0, dtype=torch.int16)
    eng.broadcast(s, 0, n, 0)
    assert torch.all(s == 3)
    # reduce-scatter ragged
    counts = [100 + 7 * i for i in range(p)]
    froms = CommUtils.getFromsFromCount(5, counts, p)
    tos = CommUtils.getTosFromCount(5, counts, p)
    t = torch.zeros(n + 100 * p)
    for i in range(p):
        t[froms[i]:tos[i]] = i + 1
    eng.reduce_scatter(t, froms, tos, Operators.Float.SUM)
    assert torch.all(t[froms[r]:tos[r]] == (r + 1) * p)
    # allgather (equal + ragged)
    for fr, to in ((CommUtils.createProcessArrayFroms(n, p), CommUtils.createProcessArrayTos(n, p)),
                   (froms, tos)):
        t = torch.full((n + 100 * p,), -1.0)
        t[fr[r]:to[r]] = r
        eng.allgather(t, fr, to)
        for i in range(p):
            assert torch.all(t[fr[i]:to[i]] == i)
    # gather / scatter / broadcast / reduce with root p-1
    root = p - 1
    fr, to = CommUtils.createProcessArrayFroms(n, p), CommUtils.createProcessArrayTos(n, p)
    t = torch.full((n,), -1.0)
    t[fr[r]:to[r]] = r
    eng.gather(t, fr, to, root)
    if r == root:
        for i in range(p):
            assert torch.all(t[fr[i]:to[i]] == i)
    t = torch.full((n,), -1.0)
    if r == root:
        for i in range(p):
            t[fr[i]:to[i]] = i
    eng.scatter(t, fr, to, root)
    assert torch.all(t[fr[r]:to[r]] == r)
    t = torch.full((n,), 1.0 if r == root else -1.0)
    eng.broadcast(t, 0, n, root)
    assert torch.all(t == 1)
    t = torch.ones(n, dtype=torch.float64)
    eng.reduce(t, 0, n, Operators.Double.SUM, None, root)
    if r == root:
        assert torch.all(t == p)
    t = torch.full((n,), 1 << r, dtype=torch.int64)
    eng.reduce(t, 0, n, Operators.Long.BITS_XOR, None, root)
    if r == root:
        assert torch.all(t == (1 << p) - 1)
    # rank-ordered custom op (non-commutative): ((r0 op r1) op r2) with x*10 + y
    from mp4x.operators import CustomOperator
    op = CustomOperator(lambda a, b: a * 10 + b, vectorized=True)
    t = torch.full((p * 3,), float(r + 1), dtype=torch.float64)
    eng.allreduce(t, 0, p * 3, op)
    expect = 0.0
    for i in range(p):
        expect = expect * 10 + (i + 1) if i else 1.0
    assert torch.all(t == expect), (t, expect)
    return dict(eng.stats)


@pytest.mark.parametrize("p", [2, 3, 4])
@pytest.mark.parametrize("algo", ["rccl", "a2a", "rhd", "composite"])
def test_device_engine_gloo(p, algo):
    res, code, _ = run_ranks(p, engine_matrix, (algo,), timeout=180)
    st = res[0]
    if algo == "rhd":                            # forced RHD takes every op (K1 combines)
        assert st.get("allreduce.rhd", 0) >= 3
        return
    if algo == "composite":                      # reference schedules: scatter+AG, RS+gather
        assert st.get("broadcast.composite", 0) >= 1 and st.get("reduce.a2a", 0) >= 1
        return
    assert st.get("allreduce.a2a", 0) >= 2      # bitwise + int16 always take the a2a schedule
    if algo == "rccl":
        assert st.get("allreduce.rccl", 0) >= 1


def sparse_engine(comm):
    p, r = comm.getSlaveNum(), comm.getRank()
    # ids 0..29 shared, plus one unique id per rank; dim-3 float rows
    ids = torch.tensor(list(range(30)) + [1000 + r], dtype=torch.int64)
    vals = torch.ones(31, 3) * (r + 1)
    k, v = comm.allreduceSparse(ids, vals, Operators.Float.SUM)
    got = dict(zip(k.tolist(), v.tolist()))
    assert len(got) == 30 + p
    assert got[0] == [p * (p + 1) / 2] * 3 and got[1000 + r] == [r + 1.0] * 3
    u = comm.allreduceSetUnion(torch.tensor([r, 100, 100], dtype=torch.int64))
    assert sorted(u.tolist()) == sorted(set(range(p)) | {100})
    i = comm.allreduceSetIntersection(torch.tensor([5, 6, 50 + r], dtype=torch.int64))
    assert sorted(i.tolist()) == [5, 6]
    c = comm.allreduceListConcat(torch.tensor([r, r], dtype=torch.int64))
    assert c.tolist() == sum([[j, j] for j in range(p)], [])
    # Map<String, float[]> with tensor values -> device map path
    m = {f"feat{j}": torch.full((4,), float(r + 1)) for j in range(12)}
    m[f"only{r}"] = torch.ones(4)
    out = comm.allreduceMap(m, Operands.FLOAT_OPERAND(), Operators.Float.SUM)
    assert len(out) == 12 + p and torch.all(out["feat3"] == p * (p + 1) / 2) and torch.all(out[f"only{r}"] == 1)
    out2 = comm.allreduceMap(m, Operands.FLOAT_OPERAND(), Operators.Float.MAX)   # keys known now: no string sync
    assert torch.all(out2["feat0"] == p)
    # the rest of the map family through the public API (device values -> device paths)
    root = p - 1
    red = comm.reduceMap(m, Operands.FLOAT_OPERAND(), Operators.Float.SUM, root)
    if r == root:
        assert len(red) == 12 + p and torch.all(red["feat5"] == p * (p + 1) / 2)
    g = comm.gatherMap({} if r == 0 else {f"g{r}": torch.ones(2)}, Operands.FLOAT_OPERAND(), root)
    if r == root:
        assert sorted(g) == sorted(f"g{q}" for q in range(1, p))
    lst = comm.allgatherMap({f"a{r}": torch.full((2,), float(r))}, Operands.FLOAT_OPERAND())
    assert [float(d[f"a{q}"][0]) for q, d in enumerate(lst)] == [float(q) for q in range(p)]
    b = comm.broadcastMap({"z": torch.tensor([3.0, 4.0])} if r == 0 else {}, Operands.FLOAT_OPERAND(), 0)
    assert torch.equal(b["z"], torch.tensor([3.0, 4.0]))
    hb = comm.broadcastMap({"h": 1.5} if r == 0 else {}, Operands.DOUBLE_OPERAND(), 0)   # host values
    assert hb == {"h": 1.5}
    ks, vs = comm.reduceSparse(torch.tensor([1, 2], dtype=torch.int64), torch.ones(2, 3), Operators.Float.SUM, 0)
    if r == 0:
        assert ks.tolist() == [1, 2] and torch.all(vs == p)
    rsm = comm.reduceScatterMap([{f"t{j}": torch.ones(2)} for j in range(p)], Operands.FLOAT_OPERAND(),
                                Operators.Float.SUM)
    assert list(rsm) == [f"t{r}"] and torch.all(rsm[f"t{r}"] == p)
    sm = comm.scatterMap([{f"q{j}": torch.full((2,), float(j))} for j in range(p)] if r == root else [{}] * p,
                         Operands.FLOAT_OPERAND(), root)
    assert list(sm) == [f"q{r}"] and torch.all(sm[f"q{r}"] == r)
    recv, rc = comm.alltoallArray(torch.full((p, 2), float(r)), [1] * p)
    assert rc == [1] * p and recv[:, 0].tolist() == [float(q) for q in range(p)]
    return "ok"


@pytest.mark.parametrize("p", [2, 3])
def test_sparse_engine_gloo(p):
    run_ranks(p, sparse_engine, timeout=120)


# rhd is an opt-in schedule (MP4X_AUTOTUNE_EXTRA=1): these tests use it as the odd candidate
EXTRA = {"MP4X_AUTOTUNE_EXTRA": "1"}


def autotune_job(comm):
    eng = comm.device
    assert eng.algo == "auto"
    t = torch.ones(4096, dtype=torch.float32)
    res = eng.autotune_allreduce(t, Operators.Float.SUM, iters=2)
    assert set(res) == {"rccl", "a2a", "rhd"} and all(v > 0 for v in res.values())
    best = min(res, key=res.get)
    eng.stats.clear()
    x = torch.full((3000,), float(comm.getRank() + 1))     # same log2 size class as 4096 floats
    eng.allreduce(x, 0, 3000, Operators.Float.SUM)
    p = comm.getSlaveNum()
    assert torch.all(x == p * (p + 1) / 2)
    return best, dict(eng.stats)


@pytest.mark.parametrize("p", [2, 3])
def test_autotune_pins_fastest_schedule_consistently(p):
    res, code, _ = run_ranks(p, autotune_job, timeout=120, env=EXTRA)
    assert code == 0
    bests = {b for b, _ in res.values()}
    assert len(bests) == 1                      # every rank made the same decision
    best = bests.pop()
    assert all(st.get("allreduce." + best) == 1 for _, st in res.values())


def broken_candidate_job(comm, dtype_name, opname):
    """rank 1's "a2a" result is corrupted in one element: the probe catches it on that rank
    only, the verdict is agreed, and every rank rules a2a out (inf) without a hang."""
    eng = comm.device
    dt = getattr(torch, dtype_name)
    orig = eng._run_allreduce

    def sabotaged(c, view, op):
        orig(c, view, op)
        if c == "a2a" and comm.getRank() == 1:
            view[7] += 1
    eng._run_allreduce = sabotaged
    res = eng.autotune_allreduce(torch.ones(4096, dtype=dt), getattr(Operators.Float, opname), iters=1)
    eng._run_allreduce = orig
    return res


@pytest.mark.parametrize("dtype_name,opname", [("float32", "SUM"), ("bfloat16", "MAX"), ("float32", "MIN")])
def test_autotune_probe_rejects_a_wrong_schedule(dtype_name, opname):
    res, code, _ = run_ranks(3, broken_candidate_job, (dtype_name, opname), timeout=120, env=EXTRA)
    assert code == 0
    for r in res.values():
        assert r["a2a"] == float("inf") and len(r) >= 2
        assert all(v < float("inf") for c, v in r.items() if c != "a2a")   # exact on the probe pattern


def _abort_job(comm):
    t = torch.ones(64)
    comm.device.allreduce(t, 0, 64, Operators.Float.SUM)
    assert torch.all(t == comm.getSlaveNum())
    if comm.getRank() == 0:
        comm.close(1)                 # failure close: the device communicator is aborted
        assert not comm.device._owns_pg
        return "aborted"
    return "ok"


def test_failure_close_aborts_device_communicator():
    res, code, errs = run_ranks(2, _abort_job, timeout=60, expect_fail=True)
    assert res.get(0) == "aborted" and not errs
    assert code == 1                  # the master aggregates the non-zero close


def rsag_autotune_job(comm):
    eng = comm.device
    p, r = comm.getSlaveNum(), comm.getRank()
    t = torch.ones(4096, dtype=torch.float32)
    rs = eng.autotune_reduce_scatter(t, Operators.Float.SUM, iters=2)
    ag = eng.autotune_allgather(t, iters=2)
    assert set(rs) == {"rccl", "a2a"} and set(ag) == {"rccl", "p2p"}     # no IPC on CPU tensors
    eng.stats.clear()
    froms, tos, _ = CommUtils.even_split(0, 4000, p)                        # same size class
    x = torch.full((4000,), float(r + 1))
    eng.reduce_scatter(x, froms, tos, Operators.Float.SUM)
    assert torch.all(x[froms[r]:tos[r]] == p * (p + 1) / 2)
    y = torch.full((4000,), -1.0)
    y[froms[r]:tos[r]] = r
    eng.allgather(y, froms, tos)
    for j in range(p):
        assert torch.all(y[froms[j]:tos[j]] == j)
    best_rs = min(rs, key=rs.get)
    best_ag = min(ag, key=ag.get)
    return best_rs, best_ag, dict(eng.stats)


def test_rs_ag_autotune_consistent_and_applied():
    res, code, _ = run_ranks(2, rsag_autotune_job, timeout=120)
    assert code == 0
    assert len({(a, b) for a, b, _ in res.values()}) == 1
    for best_rs, best_ag, st in res.values():
        assert st.get("reduce_scatter." + ("a2a" if best_rs == "a2a" else "rccl")) == 1
        assert st.get("allgather.p2p" if best_ag == "p2p" else "allgather") == 1


def tuning_roundtrip_job(comm, path):
    import os
    eng = comm.device
    t = torch.ones(4096, dtype=torch.float32)
    eng.autotune_allreduce(t, Operators.Float.SUM, iters=1)
    eng.autotune_reduce_scatter(t, Operators.Float.SUM, iters=1)
    comm.peer_barrier()                       # rank 0 has written the table (MP4X_TUNE_FILE)
    assert os.path.exists(path)
    table = eng.tuning_table()
    before = dict(eng._tuned)
    eng._tuned.clear()
    n = eng.load_tuning(path)
    assert dict(eng._tuned) == before and n == len(table["rows"])
    bad = dict(table, topology=dict(table["topology"], p=99))
    try:
        eng.load_tuning(bad)
        raise AssertionError("foreign topology accepted")
    except Exception as e:                    # noqa: BLE001
        assert "tuning table for" in str(e)
    return n


def test_tuning_table_persists_and_reloads(tmp_path):
    path = str(tmp_path / "tune.json")
    res, code, _ = run_ranks(2, tuning_roundtrip_job, args=(path,), timeout=120, env={"MP4X_TUNE_FILE": path})
    assert code == 0 and len(set(res.values())) == 1 and res[0] >= 1


def broken_rsag_job(comm):
    """every reduce-scatter result is corrupted on rank 1 and every all-gather on rank 0: all
    candidates are ruled out on all ranks (agreed verdict, no hang) and nothing is pinned."""
    eng = comm.device
    r = comm.getRank()
    rs0, ag0 = eng.reduce_scatter, eng.allgather

    def rs(view, froms, tos, op):
        rs0(view, froms, tos, op)
        if r == 1:
            view[froms[r]] += 1

    def ag(view, froms, tos):
        ag0(view, froms, tos)
        if r == 0:
            view[-1] += 1
    eng.reduce_scatter, eng.allgather = rs, ag
    t = torch.ones(4096, dtype=torch.float32)
    a = eng.autotune_reduce_scatter(t, Operators.Float.SUM, iters=1)
    b = eng.autotune_allgather(t, iters=1)
    return a, b, dict(eng._tuned)


def test_rsag_autotune_probe_rejects_wrong_results():
    res, code, _ = run_ranks(2, broken_rsag_job, timeout=120)
    assert code == 0
    for a, b, tuned in res.values():
        assert all(v == float("inf") for v in a.values()) and all(v == float("inf") for v in b.values())
        assert not tuned


def shared_table_job(comm, path):
    """Only rank 0 can read the tuning file (rank 1's path is missing, as on a host without
    the shared filesystem): every rank must pin rank 0's table, identically."""
    import os
    if comm.getRank() != 0:
        os.environ["MP4X_TUNE_FILE"] = path + ".missing"
    eng = comm.device
    return dict(eng._tuned)


def test_tuning_table_comes_from_rank0_only(tmp_path):
    import json
    path = str(tmp_path / "tune.json")
    rows = [{"kind": "allreduce", "dtype": "float32", "op": 0, "size_class": 14, "algo": "a2a"}]
    with open(path, "w") as f:
        json.dump({"topology": {"p": 2, "device": "cpu", "backend": "gloo"}, "rows": rows}, f)
    res, code, _ = run_ranks(2, shared_table_job, args=(path,), timeout=120, env={"MP4X_TUNE_FILE": path})
    assert code == 0
    assert res[0] == res[1] and len(res[0]) == 1, res


def one_rank_raises_job(comm):
    """A schedule whose local post-check raises on ONE rank during its warm-up (after its
    transport calls completed): that rank only sets a flag, every rank still joins the same
    agreement collectives, and the schedule is ruled out everywhere (no mispaired collectives,
    no hang).  Before r2 the raising rank skipped the agreement all_reduce its peers entered."""
    eng = comm.device
    orig = eng._run_allreduce

    def flaky(c, view, op):
        orig(c, view, op)
        if c == "rhd" and comm.getRank() == 1:
            raise RuntimeError("local failure on rank 1")
    eng._run_allreduce = flaky
    res = eng.autotune_allreduce(torch.ones(4096), Operators.Float.SUM, iters=2)
    eng._run_allreduce = orig
    t = torch.ones(64)
    eng.allreduce(t, 0, 64, Operators.Float.SUM)          # the job goes on
    assert torch.all(t == comm.getSlaveNum())
    return res


def test_autotune_local_failure_is_agreed():
    res, code, _ = run_ranks(3, one_rank_raises_job, timeout=120, env=EXTRA)
    assert code == 0
    for r in res.values():
        assert r["rhd"] == float("inf") and all(v < float("inf") for c, v in r.items() if c != "rhd")


def capped_job(comm):
    """A schedule whose warm-up exceeds MP4X_AUTOTUNE_CAP_S gets no timed calls (only the two
    probe calls: warm-up and the call on the previous result)."""
    import time as _t
    eng = comm.device
    orig = eng._run_allreduce
    calls = {"rhd": 0}

    def slow(c, view, op):
        if c == "rhd":
            calls["rhd"] += 1
            _t.sleep(0.3)
        orig(c, view, op)
    eng._run_allreduce = slow
    res = eng.autotune_allreduce(torch.ones(4096), Operators.Float.SUM, iters=5)
    eng._run_allreduce = orig
    return res, calls["rhd"]


def test_autotune_wall_cap(monkeypatch):
    res, code, _ = run_ranks(2, capped_job, timeout=120, env={"MP4X_AUTOTUNE_CAP_S": "0.1", **EXTRA})
    assert code == 0
    for r, n in res.values():
        assert n == 2 and r["rhd"] >= 0.3, (r, n)    # warm-up + second probe call, no timed calls


def first_op_is_a_map_with_an_empty_rank(comm):
    """The job's FIRST device op is a map collective and rank 0's map is empty: rank 0 learns
    "device" only in the agreement round, so no rank may bootstrap the (collective) device
    engine before that round (it used to: rank 1 waited in the process-group bootstrap while
    rank 0 waited in the round)."""
    r = comm.getRank()
    assert comm._device_engine is None
    m = {} if r == 0 else {"a": torch.ones(3), f"b{r}": torch.full((3,), 2.0)}
    out = comm.allreduceMap(m, Operands.FLOAT_OPERAND(), Operators.Float.SUM)
    p = comm.getSlaveNum()
    assert torch.equal(out["a"], torch.full((3,), float(p - 1)))
    assert len(out) == 1 + (p - 1)
    out = comm.allreduceMap({"a": torch.ones(3)}, Operands.FLOAT_OPERAND(), Operators.Float.SUM)
    assert torch.equal(out["a"], torch.full((3,), float(p)))
    # the other map collectives with one empty rank (engine up by now)
    red = comm.reduceMap({} if r == 1 else {"a": torch.ones(3)}, Operands.FLOAT_OPERAND(), Operators.Float.SUM, 0)
    if r == 0:
        assert torch.equal(red["a"], torch.full((3,), float(p - 1)))
    lst = comm.allgatherMap({} if r == 1 else {f"x{r}": torch.full((3,), float(r))}, Operands.FLOAT_OPERAND())
    assert len(lst) == p and len(lst[1]) == 0 and torch.equal(lst[0]["x0"], torch.zeros(3))
    return "ok"


@pytest.mark.parametrize("p", [2, 3])
def test_first_device_op_is_a_map_with_an_empty_rank(p):
    res, code, _ = run_ranks(p, first_op_is_a_map_with_an_empty_rank, timeout=90)
    assert code == 0 and set(res.values()) == {"ok"}


def rooted_autotune_job(comm):
    """reduce / broadcast / gather / scatter autotuners: every candidate exact-probed, the
    verdict agreed, the fastest pinned (RCCL pinned explicitly) and then used."""
    eng = comm.device
    p, r = comm.getSlaveNum(), comm.getRank()
    t = torch.ones(6000, dtype=torch.float32)
    root = p - 1
    red = eng.autotune_reduce(t, Operators.Float.SUM, root=root, iters=2)
    bc = eng.autotune_broadcast(t, root=root, iters=2)
    ga = eng.autotune_gather(t, root=root, iters=2)
    sc = eng.autotune_scatter(t, root=root, iters=2)
    assert set(red) == {"rccl", "a2a"} and set(bc) == {"rccl", "composite"}   # no IPC on CPU tensors
    assert set(ga) == {"p2p"} and set(sc) == {"p2p"}
    assert all(v != float("inf") for d in (red, bc, ga, sc) for v in d.values()), (red, bc, ga, sc)
    pinned = {k[0]: v for k, v in eng._tuned.items() if isinstance(k[0], str)}
    eng.stats.clear()
    x = torch.full((5000,), float(r + 1))                       # same size class as the probe
    eng.reduce(x, 0, 5000, Operators.Float.SUM, None, root)
    ok = r != root or bool(torch.all(x == p * (p + 1) / 2))
    y = torch.arange(5000, dtype=torch.float32) if r == root else torch.zeros(5000)
    eng.broadcast(y, 0, 5000, root)
    ok = ok and bool(torch.equal(y, torch.arange(5000, dtype=torch.float32)))
    return pinned, ok, dict(eng.stats)


def test_rooted_autotuners_pin_and_apply():
    res, code, _ = run_ranks(3, rooted_autotune_job, timeout=120, env=EXTRA)   # composite is opt-in
    assert code == 0
    assert len({tuple(sorted(pin.items())) for pin, _, _ in res.values()}) == 1     # agreed
    for pin, ok, st in res.values():
        assert ok
        assert set(pin) >= {"reduce", "broadcast", "gather", "scatter"}
        assert st.get("reduce." + pin["reduce"]) == 1, st
        assert st.get("broadcast" if pin["broadcast"] == "rccl" else "broadcast.composite") == 1, st


def test_zero_copy_grid_variants_are_candidates_on_a_gpu_of_their_own(monkeypatch):
    """``ipc2z_b<N>`` (the zero-copy two-shot on N blocks) is tried for large messages when
    every rank has a GPU of its own (opt-in: MP4X_AUTOTUNE_EXTRA=1); never on a shared GPU (its
    grid is capped there anyway) or under the gloo stand-in."""
    monkeypatch.setenv("MP4X_AUTOTUNE_EXTRA", "1")
    from mp4x import Operators
    from mp4x.parallel.device_engine import ZC_GRIDS, DeviceEngine, zc_grid
    assert zc_grid("ipc2z_b64") == ("ipc2z", 64) and zc_grid("ipc2z") == ("ipc2z", 0)
    assert zc_grid("ipc2z_bx") == ("ipc2z_bx", 0) and zc_grid("rccl_c64") == ("rccl_c64", 0)
    e = object.__new__(DeviceEngine)
    e.backend, e.device, e.ipc_enabled, e._zc = "nccl", torch.device("cuda", 0), True, True
    e.ipc_twoshot_max = 16 << 20
    e.rccl_ok = lambda op, dt: True
    e._ipc_ok = lambda op, dt, nb: True

    class _Ipc:
        shared_gpu = False
    e._ipc_obj = _Ipc()
    op = Operators.Float.SUM
    big = e.allreduce_candidates(256 << 20, op, torch.float32)
    assert all(f"ipc2z_b{g}" in big for g in ZC_GRIDS) and "ipc2z" in big and "rccl" in big
    assert not any(c.startswith("ipc2z_b") for c in e.allreduce_candidates(16 << 20, op, torch.float32))
    assert all(e._algo_valid(f"ipc2z_b{g}", op, torch.float32, 256 << 20) for g in ZC_GRIDS)
    assert all(f"ipc2z_b{g}" in DeviceEngine._KNOWN_ALGOS["allreduce"] for g in ZC_GRIDS)
    e._ipc_obj.shared_gpu = True
    assert not any(c.startswith("ipc2z_b") for c in e.allreduce_candidates(256 << 20, op, torch.float32))
    e._ipc_obj.shared_gpu, e.backend = False, "gloo"
    assert not any(c.startswith("ipc2z_b") for c in e.allreduce_candidates(256 << 20, op, torch.float32))


def test_select_memo_sees_every_state_change():
    """select() memoises per call shape; a re-tune, a cleared table, a forced algorithm, IPC being
    switched off or a moved tier threshold must each change the decision at once."""
    from mp4x import Operands, Operators
    from mp4x.parallel.device_engine import DeviceEngine, _TunedTable, _tune_key
    e = object.__new__(DeviceEngine)
    e.backend, e.device, e.ipc_enabled, e._zc = "nccl", torch.device("cuda", 0), True, True
    e.ipc_twoshot_max, e.ipc_oneshot_max, e.algo, e.a2a_bytes, e.p = 16 << 20, 256 << 10, "auto", 0, 2
    e._tuned, e._sel_memo, e._select_tuned = _TunedTable(), {}, False
    op, opnd = Operators.Float.SUM, Operands.FLOAT_OPERAND()
    sel = lambda nb=4096: e.select("allreduce", nb, op, torch.float32, opnd)   # noqa: E731
    assert sel() == "ipc1" and sel() == "ipc1" and len(e._sel_memo) == 1
    e._tuned[_tune_key(torch.float32, op, 4096)] = "rccl"
    assert sel() == "rccl" and e._select_tuned
    e._tuned.clear()
    assert sel() == "ipc1" and not e._select_tuned
    e.algo = "a2a"
    assert sel() == "a2a"
    e.algo = "auto"
    e.ipc_oneshot_max = 1024
    assert sel() == "ipc2"
    e.ipc_enabled = False
    assert sel() == "rccl"
    assert e.select("allreduce", 4096, op, torch.float32, Operands.FLOAT_OPERAND(compress=True)) == "zs"
    before = e._tuned.gen
    e._tuned.update({"x": 1})
    e._tuned.pop("x")
    assert e._tuned.gen == before + 2
