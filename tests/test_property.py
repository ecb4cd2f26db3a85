"""Randomised property checks of the host engine against a NumPy reference.

Every rank draws the SAME sequence of random cases (shared seed) and can regenerate every
other rank's input from (seed, rank), so each rank checks its own result against an exact
NumPy computation: random dtypes/ops, ragged and empty ranges, random roots, p up to 8.
"""
import numpy as np
import pytest

from harness import run_ranks
from mp4x import CommUtils, Operands, Operators

KINDS = [("double", np.float64, Operands.DOUBLE_OPERAND, Operators.Double),
         ("long", np.int64, Operands.LONG_OPERAND, Operators.Long),
         ("int", np.int32, Operands.INT_OPERAND, Operators.Int),
         ("byte", np.int8, Operands.BYTE_OPERAND, Operators.Byte)]


def _input(seed, case, rank, n, dt):
    rng = np.random.default_rng([seed, case, rank])
    if np.dtype(dt).kind == "f":
        return rng.integers(-8, 8, n).astype(dt)   # exact in fp: SUM order does not matter
    return rng.integers(-50, 50, n).astype(dt)


def _ref(op, xs):
    acc = xs[0].copy()
    with np.errstate(over="ignore"):
        for x in xs[1:]:
            op.reduce_into(acc, x)
    return acc


def random_cases(comm, seed, cases):
    p, r = comm.getSlaveNum(), comm.getRank()
    rng = np.random.default_rng(seed)
    for case in range(cases):
        name, dt, mk, ops = KINDS[rng.integers(len(KINDS))]
        opname = rng.choice(["SUM", "MAX", "MIN"] + (["BITS_XOR", "BITS_OR"] if name != "double" else []))
        op = getattr(ops, opname)
        n = int(rng.integers(0, 300))
        coll = rng.choice(["allreduce", "reduce_scatter", "allgather", "gather", "scatter", "reduce", "bcast"])
        root = int(rng.integers(p))
        compress = bool(rng.integers(2))
        operand = mk(compress)
        xs = [_input(seed, case, j, n, dt) for j in range(p)]
        a = xs[r].copy()
        if coll == "allreduce":
            f = int(rng.integers(0, n + 1))
            t = int(rng.integers(f, n + 1))
            comm.allreduceArray(a, operand, op, f, t)
            exp = xs[r].copy()
            if t > f:
                exp[f:t] = _ref(op, [x[f:t] for x in xs])
            assert np.array_equal(a, exp), (case, coll)
        elif coll == "reduce_scatter":
            cuts = np.sort(rng.integers(0, n + 1, p - 1)) if p > 1 else np.array([], dtype=np.int64)
            bounds = [0] + cuts.tolist() + [n]
            counts = [bounds[i + 1] - bounds[i] for i in range(p)]
            comm.reduceScatterArray(a, operand, op, 0, counts)
            f, t = bounds[r], bounds[r + 1]
            if t > f and p > 1:
                assert np.array_equal(a[f:t], _ref(op, [x[f:t] for x in xs])), (case, coll)
        else:
            cuts = np.sort(rng.integers(0, n + 1, p - 1)) if p > 1 else np.array([], dtype=np.int64)
            bounds = [0] + cuts.tolist() + [n]
            froms, tos = bounds[:-1], bounds[1:]
            if coll == "allgather":
                comm.allgatherArray(a, operand, froms, tos)
                for j in range(p):
                    assert np.array_equal(a[froms[j]:tos[j]], xs[j][froms[j]:tos[j]]), (case, coll)
            elif coll == "gather":
                comm.gatherArray(a, operand, froms, tos, root)
                if r == root:
                    for j in range(p):
                        assert np.array_equal(a[froms[j]:tos[j]], xs[j][froms[j]:tos[j]]), (case, coll)
            elif coll == "scatter":
                comm.scatterArray(a, operand, froms, tos, root)
                assert np.array_equal(a[froms[r]:tos[r]], xs[root][froms[r]:tos[r]]), (case, coll)
            elif coll == "reduce":
                comm.reduceArray(a, operand, op, 0, n, root)
                if r == root and p > 1:
                    assert np.array_equal(a, _ref(op, xs)), (case, coll)
            else:
                comm.broadcastArray(a, operand, 0, n, root)
                assert np.array_equal(a, xs[root]), (case, coll)
    return cases


@pytest.mark.parametrize("p,seed", [(2, 11), (3, 12), (5, 13), (8, 14)])
def test_random_collectives_match_numpy(p, seed):
    res, code, _ = run_ranks(p, random_cases, (seed, 60), timeout=240, env={"MP4X_SHM": "0"})   # TCP mesh
    assert code == 0 and all(v == 60 for v in res.values())


@pytest.mark.parametrize("p,seed", [(3, 21), (8, 22)])
def test_random_collectives_shared_memory(p, seed):
    res, code, _ = run_ranks(p, random_cases, (seed, 40), timeout=240)    # /dev/shm: the same-host default
    assert code == 0


@pytest.mark.parametrize("algo,p,seed", [("ring", 4, 31), ("rhd", 3, 32), ("rhd", 6, 33), ("rhd", 7, 34),
                                         ("ring", 7, 35)])
def test_random_collectives_forced_host_allreduce_algo(algo, p, seed):
    """Both host allreduce schedules (ring / recursive halving-doubling with fold) vs NumPy."""
    res, code, _ = run_ranks(p, random_cases, (seed, 30), timeout=240, env={"MP4X_HOST_ALGO": algo, "MP4X_SHM": "0"})
    assert code == 0 and all(v == 30 for v in res.values())


def _float_allreduce_digest(comm, n):
    import hashlib
    r = comm.getRank()
    a = np.random.default_rng(r).standard_normal(n)
    comm.allreduceArray(a, Operands.DOUBLE_OPERAND(), Operators.Double.SUM, 0, n)
    return hashlib.sha1(a.tobytes()).hexdigest()


@pytest.mark.parametrize("algo,p", [("rhd", 5), ("rhd", 8), ("ring", 5)])
def test_host_allreduce_bit_identical_across_ranks(algo, p):
    res, code, _ = run_ranks(p, _float_allreduce_digest, (10_001,), timeout=120, env={"MP4X_HOST_ALGO": algo, "MP4X_SHM": "0"})
    assert code == 0 and len(set(res.values())) == 1
