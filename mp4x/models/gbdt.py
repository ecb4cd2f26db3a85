"""Data-parallel histogram GBDT — the other ytk-learn consumer of the reference
(README.md:268-280: GBDT statistics synchronised with ``allreduceArray``).

Rows are sharded over ranks.  Per tree level every rank builds the gradient / hessian
histograms ``[nodes, features, bins, 2]`` of its rows and ONE ``allreduceArray`` sums them
across the job (on GPU tensors this is RCCL / the IPC kernels; on host arrays the TCP ring).
All ranks then pick identical splits, so trees never need to be broadcast.  Works on numpy
(host) or torch tensors (CPU or GPU).  Squared loss.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List

import numpy as np

from ..operands import Operands
from ..operators import Operators


@dataclass
class Tree:
    feature: List[int] = field(default_factory=list)
    threshold: List[int] = field(default_factory=list)   # bin index: go left if bin <= threshold
    left: List[int] = field(default_factory=list)
    right: List[int] = field(default_factory=list)
    value: List[float] = field(default_factory=list)

    def predict_bins(self, B: np.ndarray) -> np.ndarray:
        out = np.empty(B.shape[0])
        for i in range(B.shape[0]):
            n = 0
            while self.left[n] >= 0:
                n = self.left[n] if B[i, self.feature[n]] <= self.threshold[n] else self.right[n]
            out[i] = self.value[n]
        return out


def quantize(X: np.ndarray, bins: int, edges=None):
    if edges is None:
        edges = [np.quantile(X[:, j], np.linspace(0, 1, bins + 1)[1:-1]) for j in range(X.shape[1])]
    B = np.stack([np.searchsorted(edges[j], X[:, j], side="right") for j in range(X.shape[1])], 1).astype(np.int32)
    return B, edges


def train_gbdt(comm, B: np.ndarray, y: np.ndarray, bins: int, trees: int = 5, depth: int = 3, lr: float = 0.3,
               lam: float = 1.0) -> List[Tree]:
    p = comm.getSlaveNum() if comm is not None else 1
    n, F = B.shape
    pred = np.zeros(n)
    out: List[Tree] = []
    for _ in range(trees):
        g = pred - y          # d/dpred 0.5 (pred - y)^2
        h = np.ones(n)
        node_of = np.zeros(n, dtype=np.int64)
        tree = Tree([-1], [-1], [-1], [-1], [0.0])
        frontier = [0]
        for level in range(depth + 1):
            k = len(frontier)
            slot = {nd: i for i, nd in enumerate(frontier)}
            sel = np.isin(node_of, frontier)
            rows = np.nonzero(sel)[0]
            # local histograms [k, F, bins, 2] -> one allreduce for the whole level
            hist = np.zeros((k, F, bins, 2))
            ks = np.array([slot[v] for v in node_of[rows]], dtype=np.int64)
            for f in range(F):
                idx = (ks * bins + B[rows, f])
                hist[:, f, :, 0] = np.bincount(idx, weights=g[rows], minlength=k * bins).reshape(k, bins)
                hist[:, f, :, 1] = np.bincount(idx, weights=h[rows], minlength=k * bins).reshape(k, bins)
            flat = hist.reshape(-1)
            if comm is not None and p > 1:
                comm.allreduceArray(flat, Operands.DOUBLE_OPERAND(), Operators.Double.SUM, 0, flat.size)
            hist = flat.reshape(k, F, bins, 2)
            new_frontier = []
            for i, nd in enumerate(frontier):
                G = hist[i, 0, :, 0].sum()
                H = hist[i, 0, :, 1].sum()
                tree.value[nd] = -G / (H + lam) * lr
                if level == depth or H < 2:
                    continue
                cg = np.cumsum(hist[i, :, :, 0], axis=1)
                ch = np.cumsum(hist[i, :, :, 1], axis=1)
                gain = cg ** 2 / (ch + lam) + (G - cg) ** 2 / (H - ch + lam) - G ** 2 / (H + lam)
                gain[:, -1] = -np.inf
                f, t = np.unravel_index(int(np.argmax(gain)), gain.shape)
                if gain[f, t] <= 1e-12:
                    continue
                li, ri = len(tree.value), len(tree.value) + 1
                for _ in range(2):
                    tree.feature.append(-1)
                    tree.threshold.append(-1)
                    tree.left.append(-1)
                    tree.right.append(-1)
                    tree.value.append(0.0)
                tree.feature[nd], tree.threshold[nd], tree.left[nd], tree.right[nd] = int(f), int(t), li, ri
                m = node_of == nd
                go_left = B[:, f] <= t
                node_of[m & go_left] = li
                node_of[m & ~go_left] = ri
                new_frontier += [li, ri]
            if not new_frontier:
                break
            frontier = new_frontier
        pred += tree.predict_bins(B)
        out.append(tree)
    return out
