"""Process-level check matrix on the host data plane (CPU, real master + p rank processes).

Port of the reference's integration "check" harness (J/check/check<type>/Process*Check.java):
deterministic inputs, exact expected values, every collective x every operand type, ragged
ranges, root != 0, p in {1, 2, 3, 4}.
"""
import numpy as np
import pytest

from harness import run_ranks
from mp4x import Operands, Operators, Mp4jException, CommUtils
from mp4x.operators import IStringOperator, IObjectOperator, CustomOperator

PRIM = {
    "double": (Operands.DOUBLE_OPERAND, np.float64, Operators.Double),
    "float": (Operands.FLOAT_OPERAND, np.float32, Operators.Float),
    "long": (Operands.LONG_OPERAND, np.int64, Operators.Long),
    "int": (Operands.INT_OPERAND, np.int32, Operators.Int),
    "short": (Operands.SHORT_OPERAND, np.int16, Operators.Short),
    "byte": (Operands.BYTE_OPERAND, np.int8, Operators.Byte),
}


def prim_matrix(comm, kind, compress, n):
    mk, dt, ops = PRIM[kind]
    operand = mk(compress)
    p, r = comm.getSlaveNum(), comm.getRank()
    root = p - 1

    # ---- allreduce SUM on a sub-range (ProcessAllReduceCheck: all ones -> p)
    a = np.full(n, 7, dt)
    a[5:n - 3] = 1
    out = comm.allreduceArray(a, operand, ops.SUM, 5, n - 3)
    assert out is a
    assert (a[5:n - 3] == p).all() and (a[:5] == 7).all() and (a[n - 3:] == 7).all()
    # MAX / MIN
    a = np.full(n, r, dt)
    comm.allreduceArray(a, operand, ops.MAX, 0, n)
    assert (a == p - 1).all()
    a = np.full(n, r + 1, dt)
    comm.allreduceArray(a, operand, ops.MIN, 0, n)
    assert (a == 1).all()

    # ---- reduce-scatter with ragged counts (ProcessReduceScatterCheck)
    counts = [max(0, n // p - 3 + 2 * i) for i in range(p)]
    frm = 2
    froms = CommUtils.getFromsFromCount(frm, counts, p)
    tos = CommUtils.getTosFromCount(frm, counts, p)
    a = np.ones(n + 3 * p, dt)
    for i in range(p):
        a[froms[i]:tos[i]] = i + 1
    comm.reduceScatterArray(a, operand, ops.SUM, frm, counts)
    assert (a[froms[r]:tos[r]] == (r + 1) * p).all()

    # ---- allgather (ProcessAllgatherCheck): owner-indexed blocks
    froms = CommUtils.createProcessArrayFroms(n, p)
    tos = CommUtils.createProcessArrayTos(n, p)
    a = np.full(n, -1, dt)
    a[froms[r]:tos[r]] = r
    comm.allgatherArray(a, operand, froms, tos)
    for i in range(p):
        assert (a[froms[i]:tos[i]] == i).all()

    # ---- gather to root (ProcessGatherCheck: root verifies arr[i] == owner(i))
    a = np.full(n, -1, dt)
    a[froms[r]:tos[r]] = r
    comm.gatherArray(a, operand, froms, tos, root)
    if r == root:
        for i in range(p):
            assert (a[froms[i]:tos[i]] == i).all()

    # ---- scatter from root
    a = np.full(n, -1, dt)
    if r == root:
        for i in range(p):
            a[froms[i]:tos[i]] = i
    comm.scatterArray(a, operand, froms, tos, root)
    assert (a[froms[r]:tos[r]] == r).all()

    # ---- broadcast (ProcessBroadcastCheck: root = 1, others = -1)
    broot = 1 % p
    for size in (3, n):
        a = np.full(size, 1 if r == broot else -1, dt)
        comm.broadcastArray(a, operand, 0, size, broot)
        assert (a == 1).all()

    # ---- reduce to root
    a = np.ones(n, dt)
    comm.reduceArray(a, operand, ops.SUM, 0, n, root)
    if r == root:
        assert (a == p).all()

    # ---- scalar forms
    assert comm.allreduce(dt(1).item(), operand, ops.SUM) == p
    v = comm.reduce(dt(2).item(), operand, ops.SUM, root)
    if r == root:
        assert v == 2 * p
    assert comm.broadcast(dt(5 if r == broot else 0).item(), operand, broot) == 5

    # ---- RPC allreduce (ProcessRpcAllReduceCheck)
    a = np.ones(17, dt)
    comm.allreduceArrayRpc(a, operand, ops.SUM)
    assert (a == p).all()
    assert comm.allreduceRpc(dt(3).item(), operand, ops.SUM) == 3 * p

    # ---- map collectives (shared keys + a per-rank unique key -(rank+1), size == objSize + p)
    obj = 40
    m = {str(k): dt(1).item() for k in range(obj)}
    m[str(-(r + 1))] = dt(1).item()
    res = comm.allreduceMap(m, operand, ops.SUM)
    assert len(res) == obj + p
    assert all(res[str(k)] == p for k in range(obj))
    assert all(res[str(-(i + 1))] == 1 for i in range(p))
    assert m[str(0)] == 1, "caller's map must not be mutated"
    red = comm.reduceMap(m, operand, ops.SUM, root)
    if r == root:
        assert len(red) == obj + p and red["0"] == p
    g = comm.gatherMap({f"r{r}": dt(r).item()}, operand, root)
    if r == root:
        assert g == {f"r{i}": i for i in range(p)}
    ag = comm.allgatherMap({f"r{r}": dt(r).item()}, operand)
    assert [list(x.keys()) for x in ag] == [[f"r{i}"] for i in range(p)]
    bm = comm.broadcastMap({str(k): dt(k % 100).item() for k in range(30)} if r == broot else {}, operand, broot)
    assert bm == {str(k): k % 100 for k in range(30)}
    sm = comm.scatterMap([{f"to{i}": dt(i).item()} for i in range(p)] if r == root else None, operand, root)
    assert sm == {f"to{r}": r}
    rs = comm.reduceScatterMap([{f"b{i}": dt(1).item(), "x": dt(1).item()} for i in range(p)], operand, ops.SUM)
    assert rs["b" + str(r)] == p and rs["x"] == p
    return "ok"


@pytest.mark.parametrize("p", [1, 2, 3, 4])
@pytest.mark.parametrize("kind", list(PRIM))
def test_primitive_matrix(p, kind):
    """The TCP mesh engine (ring / RHD / trees); same-host ranks would otherwise take /dev/shm."""
    res, code, _ = run_ranks(p, prim_matrix, (kind, False, 1001), env={"MP4X_SHM": "0"})
    assert all(v == "ok" for v in res.values())
    assert code == 0


@pytest.mark.parametrize("kind", ["double", "int"])
def test_primitive_matrix_compressed(kind):
    res, code, _ = run_ranks(3, prim_matrix, (kind, True, 513))
    assert code == 0


def string_object_matrix(comm):
    p, r = comm.getSlaveNum(), comm.getRank()
    sop = Operands.STRING_OPERAND()
    add = IStringOperator(lambda a, b: str(int(a) + int(b)))   # the reference's parse-int-add check op
    n = 37
    a = ["1"] * n
    comm.allreduceArray(a, sop, add, 0, n)
    assert a == [str(p)] * n
    froms = CommUtils.createProcessArrayFroms(n, p)
    tos = CommUtils.createProcessArrayTos(n, p)
    a = [""] * n
    a[froms[r]:tos[r]] = [f"s{r}"] * (tos[r] - froms[r])
    comm.allgatherArray(a, sop, froms, tos)
    for i in range(p):
        assert a[froms[i]:tos[i]] == [f"s{i}"] * (tos[i] - froms[i])
    assert comm.broadcast("hello" if r == 0 else "", sop, 0) == "hello"
    assert comm.allreduceRpc("2", sop, add) == str(2 * p)

    class Node:
        def __init__(self, v):
            self.v = v

    oop = Operands.OBJECT_OPERAND()
    merge = IObjectOperator(lambda x, y: Node(x.v + y.v))
    objs = [Node(1) for _ in range(9)]
    comm.allreduceArray(objs, oop, merge, 0, 9)
    assert [o.v for o in objs] == [p] * 9
    objs = [Node(r) for _ in range(9)]
    comm.reduceArray(objs, oop, merge, 0, 9, 0)
    if r == 0:
        assert [o.v for o in objs] == [sum(range(p))] * 9

    # set / list specials (checkobject/ProcessAllReduceCheck :138-257)
    s = {r, 100}
    assert comm.allreduceSetUnion(s) == set(range(p)) | {100}
    assert comm.allreduceSetIntersection({1, 2, r + 10}) == ({1, 2} if p > 1 else {1, 2, 10})
    lc = comm.allreduceListConcat([r])
    assert sorted(lc) == list(range(p))
    mu = comm.allreduceMapSetUnion({"a": {r}, "b": {0}})
    assert mu == {"a": set(range(p)), "b": {0}}
    mi = comm.allreduceMapSetIntersection({"k": {1, 2, 3 + r}})
    assert mi["k"] == ({1, 2} if p > 1 else {1, 2, 3})
    ml = comm.allreduceMapListConcat({"k": [r]})
    assert sorted(ml["k"]) == list(range(p))
    ru = comm.reduceSetUnion({r}, 0)
    if r == 0:
        assert ru == set(range(p))
    ri = comm.reduceSetIntersection({7, r}, 0)
    if r == 0:
        assert ri == ({7} if p > 1 else {7, 0})
    rl = comm.reduceListConcat([r, r], 0)
    if r == 0:
        assert sorted(rl) == sorted(list(range(p)) * 2)
    assert comm.reduceMapSetUnion({"z": {r}}, 0) is not None
    assert comm.reduceMapSetIntersection({"z": {r}}, 0) is not None
    assert comm.reduceMapListConcat({"z": [r]}, 0) is not None
    return "ok"


@pytest.mark.parametrize("p", [1, 2, 4])
def test_string_object_matrix(p):
    run_ranks(p, string_object_matrix)


def custom_and_loc_ops(comm):
    p, r = comm.getSlaveNum(), comm.getRank()
    D, L = Operators.Double, Operators.Long
    a = np.array([D.compositeDouble(float(r), r), D.compositeDouble(float(-r), r)])
    comm.allreduceArray(a, Operands.DOUBLE_OPERAND(), D.FLOAT_MAX_LOC, 0, 1)
    comm.allreduceArray(a, Operands.DOUBLE_OPERAND(), D.FLOAT_MIN_LOC, 1, 2)
    assert D.getIntLoc(a[0]) == p - 1 and D.getIntLoc(a[1]) == p - 1
    b = np.array([L.compositeLong(5, r)], dtype=np.int64)   # all ties: first argument (lowest rank wins)
    comm.allreduceArray(b, Operands.LONG_OPERAND(), L.INT_MAX_LOC, 0, 1)
    assert L.getIntVal(int(b[0])) == 5
    c = np.full(8, 1 << r, dtype=np.int32)
    comm.allreduceArray(c, Operands.INT_OPERAND(), Operators.Int.BITS_OR, 0, 8)
    assert (c == (1 << p) - 1).all()
    vec = CustomOperator(lambda x, y: x * 2 + y, vectorized=True)
    d = np.ones(6)
    comm.allreduceArray(d, Operands.DOUBLE_OPERAND(), vec, 0, 6)
    assert np.isfinite(d).all()
    # Map<String, float[]> host path (BASELINE config 4 on the CPU)
    m = {f"f{k}": np.full(4, float(r + 1), np.float32) for k in range(10)}
    out = comm.allreduceMap(m, Operands.FLOAT_OPERAND(), Operators.Float.SUM)
    assert all(np.allclose(v, p * (p + 1) / 2) for v in out.values()) and len(out) == 10
    return "ok"


@pytest.mark.parametrize("p", [2, 3])
def test_custom_and_loc_ops(p):
    run_ranks(p, custom_and_loc_ops)


def bad_args(comm):
    p = comm.getSlaveNum()
    errs = 0
    for fn in (lambda: comm.allgatherArray(np.zeros(4), Operands.DOUBLE_OPERAND(), [0], [1, 2]),
               lambda: comm.reduceScatterArray(np.zeros(4), Operands.DOUBLE_OPERAND(), Operators.Double.SUM, 0,
                                               [1] * (p + 1)),
               lambda: comm.allreduceArray(np.zeros(4), Operands.DOUBLE_OPERAND(), Operators.Double.SUM, 3, 2),
               lambda: comm.broadcastArray(np.zeros(4), Operands.DOUBLE_OPERAND(), 0, 4, p + 3)):
        try:
            fn()
        except Mp4jException:
            errs += 1
    return errs


def test_illegal_arguments_raise():
    res, _, _ = run_ranks(2, bad_args)
    assert all(v == 4 for v in res.values())


def big_ring(comm):
    n = 3_000_007
    a = np.ones(n, np.float64)
    comm.allreduceArray(a, Operands.DOUBLE_OPERAND(), Operators.Double.SUM, 0, n)
    return float(a.sum())


def test_large_allreduce_4_ranks():
    res, _, _ = run_ranks(4, big_ring, timeout=180, env={"MP4X_SHM": "0"})     # the TCP ring
    assert all(v == 4 * 3_000_007 for v in res.values())


def traced(comm):
    a = np.ones(100)
    comm.allreduceArray(a, Operands.DOUBLE_OPERAND(), Operators.Double.SUM, 0, 100)
    comm.allreduce_array(a, Operands.DOUBLE_OPERAND(), Operators.Double.SUM, 0, 100)   # snake_case alias
    rep = comm.trace_report()
    return rep["allreduceArray"]["calls"], rep["allreduceArray"]["bytes"]


def test_trace_report_counts_calls():
    res, _, _ = run_ranks(2, traced, env={"MP4X_TRACE": "1"})
    assert all(v == (2, 1600) for v in res.values())


@pytest.mark.parametrize("p", [2, 3, 4])
@pytest.mark.parametrize("kind", ["double", "int", "byte"])
def test_primitive_matrix_shared_memory_engine(p, kind):
    """Same matrix with the /dev/shm engine (C++ host runtime), the same-host default."""
    res, code, _ = run_ranks(p, prim_matrix, (kind, False, 1001))
    assert code == 0


def shm_used(comm):
    a = np.ones(300_000)
    comm.allreduceArray(a, Operands.DOUBLE_OPERAND(), Operators.Double.SUM, 0, len(a))
    return comm._shm is not None and bool((a == comm.getSlaveNum()).all())


def test_shm_engine_selected_for_large_same_host_arrays():
    res, _, _ = run_ranks(3, shm_used)
    assert all(res.values())
