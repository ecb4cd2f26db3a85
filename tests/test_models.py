"""End-to-end consumers: DP MLP (SURVEY §7.4 acceptance), DP L-BFGS and histogram GBDT
(the ytk-learn workloads of the reference's README.md:268-280) — distributed result must
match single-process training on the concatenated data."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from harness import run_ranks  # noqa: E402


def _mlp(comm, autotune=False):
    from mp4x.models.mlp import train_dp
    return train_dp(comm, steps=6, global_batch=48, autotune=autotune)


@pytest.mark.parametrize("p,autotune", [(2, False), (3, False), (2, True)])
def test_dp_mlp_matches_single_process(p, autotune):
    from mp4x.models.mlp import train_single
    ref = train_single(steps=6, global_batch=48)
    res, code, _ = run_ranks(p, _mlp, (autotune,), timeout=120)
    for r, losses in res.items():
        np.testing.assert_allclose(losses, ref, rtol=2e-5, atol=1e-6)


def _data(n=600, d=8, seed=3):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, d))
    w = rng.normal(size=d)
    y = (X @ w + 0.3 * rng.normal(size=n) > 0).astype(np.float64)
    return X, y


def _lbfgs(comm):
    from mp4x.models.lbfgs import train_lbfgs
    X, y = _data()
    p, r = comm.getSlaveNum(), comm.getRank()
    rows = np.array_split(np.arange(len(y)), p)[r]
    w, hist = train_lbfgs(comm, X[rows], y[rows], n_total=len(y))
    return w


def test_dp_lbfgs_matches_single():
    from mp4x.models.lbfgs import train_lbfgs
    X, y = _data()
    w_ref, _ = train_lbfgs(None, X, y, n_total=len(y))
    res, _, _ = run_ranks(3, _lbfgs, timeout=120)
    for w in res.values():
        np.testing.assert_allclose(w, w_ref, rtol=1e-6, atol=1e-8)


def _gbdt(comm):
    from mp4x.models.gbdt import quantize, train_gbdt
    rng = np.random.default_rng(5)
    X = rng.normal(size=(900, 5))
    y = np.sin(X[:, 0]) + X[:, 1] ** 2 + 0.1 * rng.normal(size=900)
    B, _ = quantize(X, 16)
    p, r = comm.getSlaveNum(), comm.getRank()
    rows = np.array_split(np.arange(900), p)[r]
    trees = train_gbdt(comm, B[rows], y[rows], 16, trees=4, depth=3)
    return [(t.feature, t.threshold, np.round(t.value, 10).tolist()) for t in trees]


def test_dp_gbdt_matches_single():
    from mp4x.models.gbdt import quantize, train_gbdt
    rng = np.random.default_rng(5)
    X = rng.normal(size=(900, 5))
    y = np.sin(X[:, 0]) + X[:, 1] ** 2 + 0.1 * rng.normal(size=900)
    B, _ = quantize(X, 16)
    ref = train_gbdt(None, B, y, 16, trees=4, depth=3)
    ref = [(t.feature, t.threshold, np.round(t.value, 10).tolist()) for t in ref]
    res, _, _ = run_ranks(3, _gbdt, timeout=120)
    for trees in res.values():
        for (f, t, v), (rf, rt, rv) in zip(trees, ref):
            assert f == rf and t == rt
            np.testing.assert_allclose(v, rv, rtol=1e-8, atol=1e-10)
