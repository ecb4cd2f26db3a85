"""Columnar host allreduceMap (mp4x/parallel/hostmap.py) against a plain-Python reference,
plus the RowMap mapping semantics."""
import numpy as np
import pytest

from harness import run_ranks
from mp4x.parallel.hostmap import RowMap, _group_reduce


def test_rowmap_behaves_like_a_dict():
    rows = np.arange(12, dtype=np.float32).reshape(3, 4)
    m = RowMap(["a", "b", "c"], rows)
    assert len(m) == 3 and list(m) == ["a", "b", "c"] and not m.index_built
    assert [k for k, _ in m.items()] == ["a", "b", "c"] and len(m.items()) == 3
    assert np.array_equal(np.stack(list(m.values())), rows)
    assert not m.index_built                      # iteration never builds the index
    assert np.array_equal(m["b"], rows[1]) and "c" in m and "z" not in m and m.index_built
    assert m.get("z") is None
    m["d"] = np.ones(4, dtype=np.float32)        # structural change -> plain dict inside
    del m["a"]
    assert sorted(m) == ["b", "c", "d"] and m.columns() is None
    assert dict(m).keys() == {"b", "c", "d"}


def test_group_reduce_rank_order_and_dtype():
    from mp4x import Operators
    keys = ["x", "y", "x", "z", "y", "x"]
    rows = np.array([1, 2, 3, 4, 5, 6], dtype=np.int16)
    k, v = _group_reduce(keys, rows, Operators.Short.SUM)
    assert k == ["x", "y", "z"] and v.tolist() == [10, 7, 4] and v.dtype == np.int16
    k, v = _group_reduce(keys, rows, Operators.Short.MAX)
    assert v.tolist() == [6, 5, 4]


def _fn(comm, kind, compress):
    from mp4x import Operands, Operators
    r, p = comm.getRank(), comm.getSlaveNum()
    rng = np.random.default_rng(r)
    keys = [f"k{i}" for i in rng.choice(300, size=120, replace=False)] + [f"own{r}_{i}" for i in range(7)]
    if r == 1:
        keys = []                                 # an empty map on one rank
    if kind == "vec":
        m = {k: rng.integers(-5, 5, size=3).astype(np.float64) for k in keys}
        out = comm.allreduceMap(m, Operands.DOUBLE_OPERAND(compress), Operators.Double.SUM)
        mx = comm.allreduceMap(m, Operands.DOUBLE_OPERAND(compress), Operators.Double.MAX)
        return ({k: out[k].tolist() for k in out}, {k: mx[k].tolist() for k in mx}, m)
    m = {k: int(rng.integers(-5, 5)) for k in keys}
    out = comm.allreduceMap(m, Operands.INT_OPERAND(compress), Operators.Int.SUM)
    mx = comm.allreduceMap(m, Operands.INT_OPERAND(compress), Operators.Int.MIN)
    return dict(out), dict(mx), m


@pytest.mark.parametrize("kind,compress,p", [("vec", False, 3), ("scalar", False, 4), ("vec", True, 4),
                                             ("scalar", True, 2)])
def test_columnar_allreduce_map_matches_reference(kind, compress, p):
    res, _, _ = run_ranks(p, _fn, args=(kind, compress), timeout=120)
    inputs = [res[r][2] for r in range(p)]
    exp_sum, exp_ext = {}, {}
    for d in inputs:                              # rank-order fold, like the reference
        for k, v in d.items():
            v = np.asarray(v, dtype=np.float64)
            if k in exp_sum:
                exp_sum[k] = exp_sum[k] + v
                exp_ext[k] = np.maximum(exp_ext[k], v) if kind == "vec" else np.minimum(exp_ext[k], v)
            else:
                exp_sum[k], exp_ext[k] = v, v
    for r in range(p):
        got_sum, got_ext, _ = res[r]
        assert set(got_sum) == set(exp_sum) and set(got_ext) == set(exp_ext)
        for k in exp_sum:
            assert np.array_equal(np.asarray(got_sum[k]), exp_sum[k]), (r, k)
            assert np.array_equal(np.asarray(got_ext[k]), exp_ext[k]), (r, k)


def _chain_fn(comm):
    # a RowMap result goes straight into the next collective (no per-entry walk)
    from mp4x import Operands, Operators
    m = {f"k{i}": np.full(2, 1.0, dtype=np.float32) for i in range(50)}
    a = comm.allreduceMap(m, Operands.FLOAT_OPERAND(), Operators.Float.SUM)
    b = comm.allreduceMap(a, Operands.FLOAT_OPERAND(), Operators.Float.SUM)
    return type(a).__name__, {k: b[k].tolist() for k in b}


def test_rowmap_result_feeds_the_next_call():
    res, _, _ = run_ranks(3, _chain_fn, timeout=60)
    for r, (tname, b) in res.items():
        assert tname == "RowMap"
        assert len(b) == 50 and all(v == [9.0, 9.0] for v in b.values())
