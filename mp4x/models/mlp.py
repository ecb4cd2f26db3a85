"""Minimal end-to-end slice: a 2-layer MLP trained data-parallel with mp4x.

Each rank trains on its shard of a synthetic regression batch; gradients are synchronised
by :class:`~mp4x.models.ddp.GradientSynchronizer` (bucketed allreduce, overlapped with
backward on GPUs).  Acceptance: the loss curve matches single-process training on the
concatenated batch within fp tolerance (tests/test_models.py).
"""
from __future__ import annotations

from typing import List

import torch

from .ddp import GradientSynchronizer


class MLP(torch.nn.Module):
    def __init__(self, din: int = 64, hidden: int = 256, dout: int = 16):
        super().__init__()
        self.fc1 = torch.nn.Linear(din, hidden)
        self.fc2 = torch.nn.Linear(hidden, dout)

    def forward(self, x):
        return self.fc2(torch.relu(self.fc1(x)))


def synthetic_batch(step: int, global_batch: int, din: int, dout: int, device, seed: int = 7):
    g = torch.Generator(device="cpu").manual_seed(seed * 1000 + step)
    x = torch.randn(global_batch, din, generator=g)
    w = torch.randn(din, dout, generator=torch.Generator().manual_seed(seed))
    y = torch.tanh(x @ w)
    return x.to(device), y.to(device)


def train_dp(comm, steps: int = 5, global_batch: int = 64, din: int = 64, hidden: int = 128, dout: int = 16,
             lr: float = 0.05, device="cpu", bucket_mb: float = 0.01, autotune: bool = False) -> List[float]:
    """Returns the GLOBAL loss per step (mean over all ranks' shards)."""
    from ..operands import Operands
    from ..operators import Operators
    p, r = comm.getSlaveNum(), comm.getRank()
    torch.manual_seed(0)
    model = MLP(din, hidden, dout).to(device)
    sync = GradientSynchronizer(comm, model.parameters(), bucket_mb=bucket_mb, autotune=autotune)
    opt = torch.optim.SGD(model.parameters(), lr=lr)
    losses = []
    shard = global_batch // p
    for step in range(steps):
        x, y = synthetic_batch(step, global_batch, din, dout, device)
        xs, ys = x[r * shard:(r + 1) * shard], y[r * shard:(r + 1) * shard]
        sync.zero_grad()
        loss = torch.nn.functional.mse_loss(model(xs), ys)
        loss.backward()
        sync.finish()
        opt.step()
        lv = float(loss.detach().cpu())
        losses.append(comm.allreduce(lv, Operands.DOUBLE_OPERAND(), Operators.Double.SUM) / p if p > 1 else lv)
    return losses


def train_single(steps: int = 5, global_batch: int = 64, din: int = 64, hidden: int = 128, dout: int = 16,
                 lr: float = 0.05, device="cpu") -> List[float]:
    torch.manual_seed(0)
    model = MLP(din, hidden, dout).to(device)
    opt = torch.optim.SGD(model.parameters(), lr=lr)
    losses = []
    for step in range(steps):
        x, y = synthetic_batch(step, global_batch, din, dout, device)
        opt.zero_grad()
        loss = torch.nn.functional.mse_loss(model(x), y)
        loss.backward()
        opt.step()
        losses.append(float(loss.detach().cpu()))
    return losses
