"""Data-statistics passes of a distributed learner, the ytk-learn patterns the reference lists
as its applications (/root/reference/README.md:276-280):

1. ``count_instances``: allreduce of the instance count (and weight sum);
2. ``feature_frequency``: ``allreduceMap`` of per-feature occurrence counts (``Map<String,
   Long>`` SUM) — the vocabulary / min-frequency filter every sparse model starts from;
4. ``weighted_quantiles``: distributed weighted approximate quantiles through ``allreduceMap``
   — every rank maps (feature, rounded value) -> summed instance weight, one SUM over ranks,
   then each feature's cut points come from the merged weighted histogram (GBDT split
   candidates, feature binning).

(3 and 5 — L-BFGS and GBDT — are :mod:`mp4x.models.lbfgs` / :mod:`mp4x.models.gbdt`.)

All three work on any communicator (host maps over the TCP mesh / ``/dev/shm``; ``comm=None``
runs single-process), and the distributed result equals the single-process result on the
concatenated data (tests/test_features.py).
"""
from __future__ import annotations

import math
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

from ..operands import Operands
from ..operators import Operators

_SEP = "\x1f"      # feature / value separator inside a quantile map key


def count_instances(comm, n: int, weight_sum: float = None) -> Tuple[int, float]:
    """Global (instance count, weight sum) — two scalar allreduces (SUM)."""
    w = float(n if weight_sum is None else weight_sum)
    if comm is None or comm.getSlaveNum() == 1:
        return int(n), w
    tot = comm.allreduce(int(n), Operands.LONG_OPERAND(), Operators.Long.SUM)
    wsum = comm.allreduce(w, Operands.DOUBLE_OPERAND(), Operators.Double.SUM)
    return int(tot), float(wsum)


def feature_frequency(comm, samples: Iterable[Sequence[str]], min_count: int = 1) -> Dict[str, int]:
    """Global occurrence count of every feature name over all ranks' samples (each sample is a
    sequence of feature names; a name counts once per occurrence), filtered to ``min_count``."""
    local: Dict[str, int] = {}
    for s in samples:
        for f in s:
            local[f] = local.get(f, 0) + 1
    if comm is not None and comm.getSlaveNum() > 1:
        local = dict(comm.allreduceMap(local, Operands.LONG_OPERAND(), Operators.Long.SUM))
    return {k: int(v) for k, v in local.items() if v >= min_count}


def _round_sig(x: np.ndarray, digits: int) -> np.ndarray:
    """Round to ``digits`` significant digits (the sketch's precision: values closer than that
    share one histogram bin, which bounds the map size)."""
    x = np.asarray(x, dtype=np.float64)
    out = np.zeros_like(x)
    nz = x != 0
    mag = np.floor(np.log10(np.abs(x[nz])))
    scale = 10.0 ** (digits - 1 - mag)
    out[nz] = np.round(x[nz] * scale) / scale
    return out


def weighted_histogram(features: Dict[str, np.ndarray], weights: Optional[np.ndarray] = None,
                       digits: int = 4) -> Dict[str, float]:
    """This rank's {"feature\\x1fvalue": summed weight} map (values rounded to ``digits``
    significant digits)."""
    out: Dict[str, float] = {}
    for name, col in features.items():
        col = np.asarray(col, dtype=np.float64)
        w = np.ones_like(col) if weights is None else np.asarray(weights, dtype=np.float64)
        r = _round_sig(col, digits)
        uniq, inv = np.unique(r, return_inverse=True)
        sums = np.bincount(inv, weights=w, minlength=len(uniq))
        for v, s in zip(uniq.tolist(), sums.tolist()):
            out[f"{name}{_SEP}{v!r}"] = s
    return out


def weighted_quantiles(comm, features: Dict[str, np.ndarray], weights: Optional[np.ndarray] = None,
                       n_bins: int = 16, digits: int = 4) -> Dict[str, List[float]]:
    """Cut points of ``n_bins`` equal-weight bins per feature over all ranks' rows: ONE
    ``allreduceMap`` (SUM of weights per rounded value), then per feature the values where the
    cumulative weight crosses k/n_bins of the total (k = 1..n_bins-1), de-duplicated."""
    hist = weighted_histogram(features, weights, digits)
    if comm is not None and comm.getSlaveNum() > 1:
        hist = dict(comm.allreduceMap(hist, Operands.DOUBLE_OPERAND(), Operators.Double.SUM))
    per: Dict[str, List[Tuple[float, float]]] = {}
    for key, w in hist.items():
        name, v = key.split(_SEP, 1)
        per.setdefault(name, []).append((float(v), float(w)))
    cuts: Dict[str, List[float]] = {}
    for name in sorted(per):
        vals = sorted(per[name])
        v = np.array([a for a, _ in vals])
        cw = np.cumsum([b for _, b in vals])
        total = cw[-1]
        out: List[float] = []
        for k in range(1, n_bins):
            i = int(np.searchsorted(cw, total * k / n_bins, side="left"))
            c = float(v[min(i, len(v) - 1)])
            if c < v[-1] and (not out or c > out[-1]):   # (a cut at the maximum leaves an empty top bin)
                out.append(c)
        cuts[name] = out
    return cuts


def bin_index(col: np.ndarray, cuts: Sequence[float]) -> np.ndarray:
    """Bin of every value under ``cuts`` (values <= cuts[0] -> 0, ...)."""
    return np.searchsorted(np.asarray(cuts, dtype=np.float64), np.asarray(col, dtype=np.float64), side="left")


def quantile_error(col: np.ndarray, cuts: Sequence[float], weights: Optional[np.ndarray] = None) -> float:
    """Largest deviation of a bin's weight share from 1/(len(cuts)+1) (sketch quality)."""
    b = bin_index(col, cuts)
    w = np.ones(len(col)) if weights is None else np.asarray(weights, dtype=np.float64)
    share = np.bincount(b, weights=w, minlength=len(cuts) + 1) / w.sum()
    return float(np.abs(share - 1.0 / (len(cuts) + 1)).max()) if len(share) else math.nan
