"""Data-parallel L-BFGS logistic regression — the ytk-learn usage pattern the reference was
built for (README.md:268-280: "data-parallel L-BFGS ... allreduceArray of gradients").

Each rank owns a shard of the rows.  Every function evaluation is ONE allreduce of the packed
``[loss, grad...]`` vector (f64), so all ranks run the identical two-loop recursion and line
search and stay bit-for-bit in lockstep without broadcasting the iterate.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np

from ..operands import Operands
from ..operators import Operators


def _local_loss_grad(w: np.ndarray, X: np.ndarray, y: np.ndarray, l2: float, n_total: int, p: int):
    z = X @ w
    # logistic loss with labels in {0, 1}: log(1 + e^z) - y z   (stable form)
    loss = np.sum(np.logaddexp(0.0, z) - y * z) / n_total
    sig = 0.5 * (1.0 + np.tanh(0.5 * z))
    g = X.T @ (sig - y) / n_total
    # the L2 term is added once across the job (split over ranks)
    loss += 0.5 * l2 * float(w @ w) / p
    g += l2 * w / p
    return loss, g


def train_lbfgs(comm, X: np.ndarray, y: np.ndarray, n_total: int, l2: float = 1e-3, m: int = 7,
                iters: int = 30, tol: float = 1e-9) -> Tuple[np.ndarray, list]:
    p = comm.getSlaveNum() if comm is not None else 1
    d = X.shape[1]
    w = np.zeros(d)
    buf = np.empty(d + 1)

    def evaluate(w):
        loss, g = _local_loss_grad(w, X, y, l2, n_total, p)
        buf[0] = loss
        buf[1:] = g
        if comm is not None and p > 1:
            comm.allreduceArray(buf, Operands.DOUBLE_OPERAND(), Operators.Double.SUM, 0, d + 1)
        return float(buf[0]), buf[1:].copy()

    f, g = evaluate(w)
    S, Y = [], []
    hist = [f]
    for _ in range(iters):
        q = g.copy()
        alphas = []
        for s, yv in reversed(list(zip(S, Y))):
            a = (s @ q) / (yv @ s)
            alphas.append(a)
            q -= a * yv
        if S:
            q *= (S[-1] @ Y[-1]) / (Y[-1] @ Y[-1])
        for (s, yv), a in zip(zip(S, Y), reversed(alphas)):
            b = (yv @ q) / (yv @ s)
            q += s * (a - b)
        direction = -q
        step = 1.0
        gd = g @ direction
        if gd >= 0:
            direction, gd = -g, -(g @ g)
        while True:   # Armijo backtracking
            wn = w + step * direction
            fn, gn = evaluate(wn)
            if fn <= f + 1e-4 * step * gd or step < 1e-10:
                break
            step *= 0.5
        s, yv = wn - w, gn - g
        if s @ yv > 1e-12:
            S.append(s)
            Y.append(yv)
            if len(S) > m:
                S.pop(0)
                Y.pop(0)
        w, f, g = wn, fn, gn
        hist.append(f)
        if abs(hist[-2] - hist[-1]) < tol:
            break
    return w, hist
