"""Host map collectives: the direct mesh exchange and the reference's ring give the same maps
(exact: integer-valued floats), for allreduceMap / reduceScatterMap / allgatherMap, p = 3, 4."""
import numpy as np
import pytest

from harness import run_ranks
from mp4x import Operands, Operators


def both_algos(comm):
    from mp4x.parallel import host_engine
    r, p = comm.getRank(), comm.getSlaveNum()
    rng = np.random.default_rng(r)
    m = {f"s{i}": rng.integers(-5, 5, 3).astype(np.float64) for i in range(200)}
    m.update({f"r{r}_{i}": np.full(3, float(i)) for i in range(50)})
    scal = {f"k{i}": float(i * (r + 1)) for i in range(100)}
    out = {}
    for algo in ("ring", "direct"):
        host_engine._MAP_ALGO = algo
        ar = comm.allreduceMap(m, Operands.DOUBLE_OPERAND(), Operators.Double.SUM)
        sc = comm.allreduceMap(scal, Operands.DOUBLE_OPERAND(), Operators.Double.MAX)
        rs = comm.reduceScatterMap([{f"t{j}_{i}": np.ones(2) * (r + 1) for i in range(10)} for j in range(p)],
                                   Operands.DOUBLE_OPERAND(), Operators.Double.SUM)
        ag = comm.allgatherMap({f"a{r}": np.full(2, float(r))}, Operands.DOUBLE_OPERAND())
        out[algo] = (ar, sc, rs, ag)
    host_engine._MAP_ALGO = "auto"
    (ar1, sc1, rs1, ag1), (ar2, sc2, rs2, ag2) = out["ring"], out["direct"]
    assert ar1.keys() == ar2.keys() and all(np.array_equal(ar1[k], ar2[k]) for k in ar1)
    assert sc1 == sc2 and sc1["k3"] == 3.0 * p
    assert rs1.keys() == rs2.keys() and all(np.array_equal(rs1[k], rs2[k]) for k in rs1)
    assert np.array_equal(rs2[f"t{r}_0"], np.ones(2) * p * (p + 1) / 2)
    assert len(ag1) == len(ag2) == p and all(np.array_equal(ag2[i][f"a{i}"], np.full(2, float(i))) for i in range(p))
    return "ok"


@pytest.mark.parametrize("p", [3, 4])
def test_direct_and_ring_map_exchange_agree(p):
    res, code, _ = run_ranks(p, both_algos, timeout=120)
    assert code == 0 and set(res.values()) == {"ok"}
