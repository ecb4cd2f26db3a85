"""ThreadComm (process x thread) check matrix — port of J/check/check*/Thread*Check.java.

Expected values follow the reference checks: contributions are x slaveNum*threadNum, ranges
from CommUtils.createThreadArrayFroms/Tos, roots (rootRank, rootThreadId) != (0, 0).
BASELINE config 1 ("2-thread in-process float[1024] allreduceArray on CPU") is
``test_baseline_config1_two_threads``.
"""
import threading

import numpy as np
import pytest

from harness import run_ranks
from mp4x import CommUtils, Operands, Operators


def _run_threads(tc, fn):
    T = tc.getThreadNum()
    res = [None] * T
    errs = []

    def body(t):
        try:
            tc.setThreadId(t)
            res[t] = fn(t)
        except BaseException as e:  # noqa
            import traceback
            errs.append(traceback.format_exc())
            tc._barrier.abort()

    ths = [threading.Thread(target=body, args=(t,)) for t in range(T)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    if errs:
        raise AssertionError(errs[0])
    return res


def thread_matrix(tc, kind):
    dt, operand, ops = {"double": (np.float64, Operands.DOUBLE_OPERAND(), Operators.Double),
                        "int": (np.int32, Operands.INT_OPERAND(), Operators.Int),
                        "float": (np.float32, Operands.FLOAT_OPERAND(), Operators.Float)}[kind]
    p, r, T = tc.getSlaveNum(), tc.getRank(), tc.getThreadNum()
    n = 997
    froms = CommUtils.createThreadArrayFroms(n, p, T)
    tos = CommUtils.createThreadArrayTos(n, p, T)
    root_rank, root_tid = p - 1, T - 1

    def body(t):
        # allreduce (ThreadAllReduceCheck: ones -> p*T)
        a = np.ones(n, dt)
        tc.allreduceArray(a, operand, ops.SUM, 0, n)
        assert (a == p * T).all(), a[:4]
        # allreduce on a sub range, MAX
        a = np.full(n, r * T + t, dt)
        tc.allreduceArray(a, operand, ops.MAX, 3, n - 2)
        assert (a[3:n - 2] == p * T - 1).all() and a[0] == r * T + t
        # allgather with [p][T] ranges
        a = np.full(n, -1, dt)
        a[froms[r][t]:tos[r][t]] = r * T + t
        tc.allgatherArray(a, operand, froms, tos)
        for i in range(p):
            for j in range(T):
                assert (a[froms[i][j]:tos[i][j]] == i * T + j).all()
        # gather to (root_rank, root_tid)
        a = np.full(n, -1, dt)
        a[froms[r][t]:tos[r][t]] = r * T + t
        g = tc.gatherArray(a, operand, froms, tos, root_rank, root_tid)
        if r == root_rank and t == root_tid:
            for i in range(p):
                for j in range(T):
                    assert (g[froms[i][j]:tos[i][j]] == i * T + j).all()
        # scatter from (root_rank, root_tid)
        a = np.full(n, -1, dt)
        if r == root_rank and t == root_tid:
            for i in range(p):
                for j in range(T):
                    a[froms[i][j]:tos[i][j]] = i * T + j
        tc.scatterArray(a, operand, froms, tos, root_rank, root_tid)
        assert (a[froms[r][t]:tos[r][t]] == r * T + t).all()
        # broadcast (root thread value 1, others -1)
        a = np.full(n, 1 if (r == root_rank and t == root_tid) else -1, dt)
        tc.broadcastArray(a, operand, 0, n, root_rank, root_tid)
        assert (a == 1).all()
        # reduce-scatter with [p][T] counts (ThreadReduceScatterCheck)
        counts = [[(tos[i][j] - froms[i][j]) for j in range(T)] for i in range(p)]
        a = np.ones(n, dt)
        tc.reduceScatterArray(a, operand, ops.SUM, 0, counts)
        assert (a[froms[r][t]:tos[r][t]] == p * T).all()
        # reduce to root
        a = np.ones(n, dt)
        tc.reduceArray(a, operand, ops.SUM, 0, n, root_rank, root_tid)
        if r == root_rank and t == root_tid:
            assert (a == p * T).all()
        # scalars
        assert tc.allreduce(dt(1).item(), operand, ops.SUM) == p * T
        v = tc.reduce(dt(1).item(), operand, ops.SUM, root_rank, root_tid)
        if r == root_rank and t == root_tid:
            assert v == p * T
        assert tc.broadcast(dt(9 if (r == root_rank and t == root_tid) else 0).item(), operand,
                            root_rank, root_tid) == 9
        # rpc allreduce
        a = np.ones(11, dt)
        tc.allreduceArrayRpc(a, operand, ops.SUM)
        assert (a == p * T).all()
        assert tc.allreduceRpc(dt(2).item(), operand, ops.SUM) == 2 * p * T
        # maps: shared keys + per (rank, thread) unique key
        m = {str(k): dt(1).item() for k in range(20)}
        m[f"u{r}_{t}"] = dt(1).item()
        res = tc.allreduceMap(m, operand, ops.SUM)
        assert len(res) == 20 + p * T and res["0"] == p * T
        red = tc.reduceMap(m, operand, ops.SUM, root_rank, root_tid)
        if r == root_rank and t == root_tid:
            assert red["0"] == p * T and len(red) == 20 + p * T
        else:
            assert red is None
        ag = tc.allgatherMap({f"k{r}_{t}": dt(1).item()}, operand)
        assert len(ag) == p and set(ag[r].keys()) == {f"k{r}_{j}" for j in range(T)}
        gm = tc.gatherMap({f"k{r}_{t}": dt(1).item()}, operand, root_rank, root_tid)
        if r == root_rank and t == root_tid:
            assert len(gm) == p * T
        bm = tc.broadcastMap({"x": dt(3).item()} if (r == root_rank and t == root_tid) else {}, operand,
                             root_rank, root_tid)
        assert bm == {"x": 3}
        lists = [[{f"s{i}_{j}": dt(i * T + j).item()} for j in range(T)] for i in range(p)] \
            if (r == root_rank and t == root_tid) else None
        sm = tc.scatterMap(lists, operand, root_rank, root_tid)
        assert sm == {f"s{r}_{t}": r * T + t}
        rsl = [[{"c": dt(1).item(), f"o{i}_{j}": dt(1).item()} for j in range(T)] for i in range(p)]
        rs = tc.reduceScatterMap(rsl, operand, ops.SUM)
        assert rs["c"] == p * T and rs[f"o{r}_{t}"] == p * T
        # set/list specials
        assert tc.allreduceSetUnion({r * T + t}) == set(range(p * T))
        assert sorted(tc.allreduceListConcat([r * T + t])) == list(range(p * T))
        assert tc.allreduceSetIntersection({1, 2, 100 + r * T + t}) == ({1, 2} if p * T > 1 else {1, 2, 100})
        # *Process pass-throughs from one thread (checkbyte/ThreadAllReduceCheck :156-241)
        if t == 0:
            b = np.ones(5, dt)
            tc.allreduceArrayProcess(b, operand, ops.SUM, 0, 5)
            assert (b == p).all()
            assert tc.allreduceProcess(dt(1).item(), operand, ops.SUM) == p
        tc.barrier()
        return "ok"

    return _run_threads(tc, body)


@pytest.mark.parametrize("p,T", [(1, 1), (1, 3), (2, 2), (3, 2), (2, 4)])
@pytest.mark.parametrize("kind", ["double", "int"])
def test_thread_matrix(p, T, kind):
    res, code, _ = run_ranks(p, thread_matrix, (kind,), kind="thread", threads=T, timeout=180)
    assert code == 0 and all(v == ["ok"] * T for v in res.values())


def config1(tc):
    def body(t):
        a = np.full(1024, float(t + 1), np.float32)
        tc.allreduceArray(a, Operands.FLOAT_OPERAND(), Operators.Float.SUM, 0, 1024)
        return float(a[0]), float(a[-1])
    return _run_threads(tc, body)


def test_baseline_config1_two_threads():
    """BASELINE config 1: 2-thread in-process float[1024] allreduceArray on CPU."""
    res, code, _ = run_ranks(1, config1, kind="thread", threads=2)
    assert res[0] == [(3.0, 3.0), (3.0, 3.0)]


def stress(tc, iters):
    """Race screen: many back-to-back mixed collectives from every thread (no sleeps)."""
    p, r, T = tc.getSlaveNum(), tc.getRank(), tc.getThreadNum()

    def body(t):
        rng = np.random.default_rng(1234)          # same op sequence on every thread / rank
        for it in range(iters):
            k = int(rng.integers(4))
            n = int(rng.integers(1, 64))
            if k == 0:
                a = np.full(n, float(it + t), np.float64)
                tc.allreduceArray(a, Operands.DOUBLE_OPERAND(), Operators.Double.SUM, 0, n)
                assert (a == sum(it + j for j in range(T)) * p).all()
            elif k == 1:
                v = tc.allreduce(it * 10 + t + r, Operands.INT_OPERAND(), Operators.Int.MAX)
                assert v == it * 10 + (T - 1) + (p - 1)
            elif k == 2:
                m = tc.allreduceMap({"k": 1, f"t{t}r{r}": it}, Operands.INT_OPERAND(), Operators.Int.SUM)
                assert m["k"] == p * T and len(m) == 1 + p * T
            else:
                a = np.full(n, -1.0)
                a[:] = 5.0 if (r == 0 and t == 0) else -1.0
                tc.broadcastArray(a, Operands.DOUBLE_OPERAND(), 0, n, 0, 0)
                assert (a == 5.0).all()
        return True

    return _run_threads(tc, body)


def test_thread_stress_interleaved_collectives():
    res, code, _ = run_ranks(2, stress, (150,), kind="thread", threads=4, timeout=240)
    assert code == 0 and all(all(v) for v in res.values())


def _process_passthroughs(tc):
    """Thread 0 of every process drives every ``XProcess`` pass-through (checkbyte/Thread*Check
    :156-241 pattern); the other threads only join the final thread barrier."""
    p, r, T = tc.getSlaveNum(), tc.getRank(), tc.getThreadNum()

    def body(t):
        if t == 0:
            D, ops = Operands.DOUBLE_OPERAND(), Operators.Double
            n = 40
            fr = CommUtils.createProcessArrayFroms(n, p)
            to = CommUtils.createProcessArrayTos(n, p)
            a = np.full(n, -1.0)
            a[fr[r]:to[r]] = r
            tc.gatherArrayProcess(a, D, fr, to, 0)
            if r == 0:
                assert all((a[fr[i]:to[i]] == i).all() for i in range(p))
            a = np.full(n, -1.0)
            a[fr[r]:to[r]] = r
            tc.allgatherArrayProcess(a, D, fr, to)
            assert all((a[fr[i]:to[i]] == i).all() for i in range(p))
            a = np.arange(n, dtype=np.float64) if r == 0 else np.zeros(n)
            tc.scatterArrayProcess(a, D, fr, to, 0)
            assert (a[fr[r]:to[r]] == np.arange(fr[r], to[r])).all()
            a = np.full(n, 1.0 if r == 0 else 0.0)
            tc.broadcastArrayProcess(a, D, 0, n, 0)
            assert (a == 1).all()
            assert tc.broadcastProcess(7.0 if r == 0 else 0.0, D, 0) == 7.0
            a = np.ones(n)
            tc.reduceScatterArrayProcess(a, D, ops.SUM, 0, [t_ - f_ for f_, t_ in zip(fr, to)])
            assert (a[fr[r]:to[r]] == p).all()
            a = np.ones(n)
            tc.reduceArrayProcess(a, D, ops.SUM, 0, n, 0)
            if r == 0:
                assert (a == p).all()
            assert tc.reduceProcess(1.0, D, ops.SUM, 0) == p or r != 0
            a = np.ones(n)
            tc.allreduceArrayProcess(a, D, ops.MAX, 0, n)
            assert (a == 1).all()
            a = np.ones(8)
            tc.allreduceArrayRpcProcess(a, D, ops.SUM)
            assert (a == p).all()
            assert tc.allreduceRpcProcess(2.0, D, ops.SUM) == 2.0 * p
            m = {"k": 1.0, f"u{r}": 1.0}
            assert tc.allreduceMapProcess(m, D, ops.SUM)["k"] == p
            got = tc.reduceMapProcess(m, D, ops.SUM, 0)
            if r == 0:
                assert got["k"] == p and len(got) == 1 + p
            g = tc.gatherMapProcess({f"g{r}": 1.0}, D, 0)
            if r == 0:
                assert len(g) == p
            lst = tc.allgatherMapProcess({f"a{r}": float(r)}, D)
            assert [d[f"a{i}"] for i, d in enumerate(lst)] == [float(i) for i in range(p)]
            b = tc.broadcastMapProcess({"b": 3.0} if r == 0 else {}, D, 0)
            assert b == {"b": 3.0}
            sm = tc.scatterMapProcess([{f"s{i}": float(i)} for i in range(p)] if r == 0 else None, D, 0)
            assert sm == {f"s{r}": float(r)}
            rs = tc.reduceScatterMapProcess([{f"x{i}": 1.0} for i in range(p)], D, ops.SUM)
            assert rs == {f"x{r}": float(p)}
            assert tc.allreduceSetUnionProcess({r}) == set(range(p))
            assert tc.allreduceSetIntersectionProcess({r, 99}) == ({99} if p > 1 else {r, 99})
            assert sorted(tc.allreduceListConcatProcess([r])) == list(range(p))
            u = tc.reduceSetUnionProcess({r}, 0)
            if r == 0:
                assert u == set(range(p))
            mu = tc.allreduceMapSetUnionProcess({"k": {r}})
            assert mu["k"] == set(range(p))
        tc.threadBarrier()
        return True

    return _run_threads(tc, body)


@pytest.mark.parametrize("p", [2, 3])
def test_every_process_passthrough_from_thread0(p):
    res, code, _ = run_ranks(p, _process_passthroughs, kind="thread", threads=2, timeout=120)
    assert code == 0 and len(res) == p


def tensor_maps(tc):
    """Thread-mode map collectives with TENSOR values (CPU tensors here; the GPU twin is in
    test_thread_device_gpu.py): the thread phase reduces shared keys with one stacked reduce."""
    import torch

    p, r, T = tc.getSlaveNum(), tc.getRank(), tc.getThreadNum()

    def body(t):
        ops = Operators.Float
        m = {"shared": torch.full((4,), float(t + 1)), f"u{r}_{t}": torch.full((4,), 1.0),
             f"proc{r}": torch.full((4,), 2.0)}
        res = tc.allreduceMap(m, Operands.FLOAT_OPERAND(), ops.SUM)
        assert len(res) == 1 + p * T + p
        assert torch.equal(res["shared"], torch.full((4,), float(p * T * (T + 1) // 2)))
        assert all(torch.equal(res[f"u{i}_{j}"], torch.ones(4)) for i in range(p) for j in range(T))
        assert all(torch.equal(res[f"proc{i}"], torch.full((4,), 2.0 * T)) for i in range(p))
        mx = tc.allreduceMap({"k": torch.tensor([float(r * T + t), -float(r * T + t)])},
                             Operands.FLOAT_OPERAND(), ops.MAX)
        assert torch.equal(mx["k"], torch.tensor([float(p * T - 1), 0.0]))
        red = tc.reduceMap({"k": torch.full((3,), 1.0)}, Operands.FLOAT_OPERAND(), ops.SUM, p - 1, T - 1)
        if r == p - 1 and t == T - 1:
            assert torch.equal(red["k"], torch.full((3,), float(p * T)))
        return "ok"
    return _run_threads(tc, body)


@pytest.mark.parametrize("p,T", [(1, 3), (2, 2)])
def test_thread_tensor_maps(p, T):
    res, code, _ = run_ranks(p, tensor_maps, (), kind="thread", threads=T, timeout=180)
    assert code == 0 and all(v == ["ok"] * T for v in res.values())
