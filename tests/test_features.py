"""The ytk-learn data-statistics passes (mp4x/models/features.py; reference README.md:276-280):
instance counts, feature frequencies through allreduceMap, distributed weighted approximate
quantiles through allreduceMap — the distributed result equals the single-process result on
the concatenated data."""
import numpy as np
import pytest

from harness import run_ranks


def _data(r, n=400):
    rng = np.random.default_rng(10 + r)
    feats = {"age": rng.normal(40, 12, n), "score": rng.exponential(3.0, n), "flag": rng.integers(0, 3, n) * 1.0}
    w = rng.choice([0.5, 1.0, 2.0], n)                      # exact binary sums in any order
    samples = [[f"f{int(x)}" for x in rng.zipf(1.6, 5) if x < 500] for _ in range(n)]
    return feats, w, samples


def _stats(comm):
    from mp4x.models.features import count_instances, feature_frequency, weighted_quantiles
    feats, w, samples = _data(comm.getRank())
    n, ws = count_instances(comm, len(w), float(w.sum()))
    freq = feature_frequency(comm, samples, min_count=3)
    cuts = weighted_quantiles(comm, feats, w, n_bins=8)
    return n, ws, freq, cuts


@pytest.mark.parametrize("p", [2, 3])
def test_distributed_stats_match_single_process(p):
    from mp4x.models.features import count_instances, feature_frequency, quantile_error, weighted_quantiles
    parts = [_data(r) for r in range(p)]
    feats = {k: np.concatenate([f[k] for f, _, _ in parts]) for k in parts[0][0]}
    w = np.concatenate([x for _, x, _ in parts])
    samples = sum((s for _, _, s in parts), [])
    ref_n, ref_w = count_instances(None, len(w), float(w.sum()))
    ref_freq = feature_frequency(None, samples, min_count=3)
    ref_cuts = weighted_quantiles(None, feats, w, n_bins=8)
    res, _, _ = run_ranks(p, _stats, timeout=120)
    assert len(res) == p
    for n, ws, freq, cuts in res.values():
        assert (n, ws) == (ref_n, ref_w)
        assert freq == ref_freq and min(freq.values()) >= 3
        assert cuts == ref_cuts
    # the sketch is a real quantile: every bin holds ~1/8 of the weight (4 significant digits)
    assert quantile_error(feats["age"], ref_cuts["age"], w) < 0.02
    assert ref_cuts["flag"] == [0.0, 1.0]                     # 3 distinct values -> 2 cuts


def test_rounding_bounds_the_map():
    from mp4x.models.features import weighted_histogram
    x = np.linspace(1.0, 1.001, 10000)
    h = weighted_histogram({"x": x}, digits=4)
    assert len(h) <= 3 and abs(sum(h.values()) - 10000) < 1e-9
