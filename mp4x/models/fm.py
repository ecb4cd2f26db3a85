"""Factorization machine trained data-parallel with SPARSE gradient sync — the sparse-model
pattern behind the reference's map collectives (ytk-learn's FM / FFM family; the map API of
ProcessCommSlave.java:2053-2088 is what carries their per-feature statistics).

Per step every rank runs forward/backward on its shard; the embedding tables (``w`` linear
weights, ``v`` factor rows) produce sparse gradients: only the feature rows present in the
shard.  Both tables' rows are concatenated into one ``[n_touched, 1 + k]`` tensor and synced
with ONE ``allreduceSparse`` (K4b owner partition + ragged all-to-all / IPC copy plan + K5
reduce-by-key + all-gather on the GPU; ``keyBits`` = the vocabulary's bit width, so the radix
sort covers only those bits).  The update then touches only the union of rows any rank saw
(sparse SGD or Adagrad), exactly like a single process on the concatenated batch.
"""
from __future__ import annotations

from typing import List, Tuple

import torch

from ..operands import Operands
from ..operators import Operators


class FM(torch.nn.Module):
    """Binary-feature FM: y = w0 + sum_i w_i + 1/2 sum_f ((sum_i v_if)^2 - sum_i v_if^2) over
    the active feature ids of an instance."""

    def __init__(self, vocab: int, k: int = 8, seed: int = 0):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        self.w0 = torch.nn.Parameter(torch.zeros(()))
        self.w = torch.nn.Embedding(vocab, 1, sparse=True)
        self.v = torch.nn.Embedding(vocab, k, sparse=True)
        with torch.no_grad():
            self.w.weight.zero_()
            self.v.weight.copy_(torch.randn(vocab, k, generator=g) * 0.05)

    def forward(self, idx: torch.Tensor) -> torch.Tensor:
        e = self.v(idx)                                              # [n, nnz, k]
        inter = 0.5 * (e.sum(1).square() - e.square().sum(1)).sum(1)
        return self.w0 + self.w(idx).sum((1, 2)) + inter


def synthetic_data(n: int, vocab: int, nnz: int, seed: int = 3) -> Tuple[torch.Tensor, torch.Tensor]:
    """``n`` instances of ``nnz`` distinct-ish Zipf-distributed feature ids and 0/1 labels from a
    hidden FM (synthetic: no dataset download)."""
    g = torch.Generator().manual_seed(seed)
    ranks = torch.arange(1, vocab + 1, dtype=torch.float64)
    probs = (1.0 / ranks ** 1.1)
    idx = torch.multinomial(probs.expand(n, vocab), nnz, replacement=False, generator=g)
    truth = FM(vocab, 4, seed=seed + 1)
    with torch.no_grad():
        truth.w.weight.copy_(torch.randn(vocab, 1, generator=g) * 0.5)
        truth.v.weight.mul_(10.0)
        y = (torch.sigmoid(truth(idx)) > torch.rand(n, generator=g)).float()
    return idx, y


def _sparse_rows(model: FM) -> Tuple[torch.Tensor, torch.Tensor]:
    """(ids, [n, 1 + k] rows) of the two tables' sparse gradients (same touched ids)."""
    gw = model.w.weight.grad.coalesce()
    gv = model.v.weight.grad.coalesce()
    ids = gw.indices()[0]
    return ids, torch.cat([gw.values(), gv.values()], 1)


def _apply(model: FM, ids: torch.Tensor, rows: torch.Tensor, g0: torch.Tensor, lr: float, state: dict,
           adagrad: bool) -> None:
    with torch.no_grad():
        if adagrad:
            acc = state.setdefault("acc", torch.zeros(model.v.weight.shape[0], rows.shape[1], dtype=rows.dtype,
                                                      device=rows.device))
            acc[ids] += rows.square()
            step = rows / (acc[ids].sqrt() + 1e-8)
        else:
            step = rows
        model.w.weight[ids] -= lr * step[:, :1]
        model.v.weight[ids] -= lr * step[:, 1:]
        model.w0 -= lr * g0


def train_fm(comm, steps: int = 5, global_batch: int = 256, vocab: int = 2000, nnz: int = 12, k: int = 8,
             lr: float = 0.05, adagrad: bool = True, device="cpu") -> List[float]:
    """DP training; returns the GLOBAL mean log-loss per step.  ``comm=None``: one process on
    the whole batch (the reference trajectory)."""
    p = 1 if comm is None else comm.getSlaveNum()
    r = 0 if comm is None else comm.getRank()
    idx, y = synthetic_data(steps * global_batch, vocab, nnz)
    model = FM(vocab, k).to(device)
    state: dict = {}
    shard = global_batch // p
    bits = max(1, (vocab - 1).bit_length())
    losses = []
    for s in range(steps):
        lo = s * global_batch + r * shard
        xb, yb = idx[lo:lo + shard].to(device), y[lo:lo + shard].to(device)
        model.zero_grad(set_to_none=True)
        loss = torch.nn.functional.binary_cross_entropy_with_logits(model(xb), yb, reduction="sum") / global_batch
        loss.backward()
        ids, rows = _sparse_rows(model)
        g0 = model.w0.grad.detach().clone().reshape(1)
        lv = float(loss.detach().cpu())
        if p > 1:
            ids, rows = comm.allreduceSparse(ids, rows, Operators.Float.SUM, keyBits=bits)
            g0 = comm.allreduceArray(g0, Operands.FLOAT_OPERAND(), Operators.Float.SUM, 0, 1)
            lv = comm.allreduce(lv, Operands.DOUBLE_OPERAND(), Operators.Double.SUM)
        _apply(model, ids, rows, g0[0], lr, state, adagrad)
        losses.append(lv)
    return losses
