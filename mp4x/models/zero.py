"""ZeRO-style sharded optimizer: BASELINE config 3's reduceScatter + allgather pattern inside a
training loop (the reference has no optimizer; its ``reduceScatterArray`` / ``allgatherArray``,
ProcessCommSlave.java:436-560 / :1096-1150, are the collectives this is built from).

Every trainable parameter of one dtype lives in ONE flat arena (``param.data`` is a view), and
its gradient in a second arena (``param.grad`` is a view, autograd accumulates into it in place).
Both arenas are padded to a multiple of ``p`` 16-byte vectors, so rank ``r`` owns the contiguous,
16-byte-aligned slice ``[r*n/p, (r+1)*n/p)`` of each.  A step is:

1. ``reduceScatterArray`` on the gradient arena — rank r ends up with the reduced gradient of
   its slice only (1/p of the bytes of an allreduce on every link);
2. the 1/p average and optional global-norm clipping on the slice (the norm is one 1-element
   allreduce; the clip coefficient stays on the device, no host sync);
3. the inner optimizer (any ``torch.optim`` class, elementwise ones such as AdamW / SGD give
   the same trajectory as unsharded training) steps the slice's master copy — fp32 for bf16 /
   fp16 parameters, an alias of the slice itself for fp32 / fp64 ones — so optimizer state is
   1/p per rank;
4. ``allgatherArray`` on the parameter arena publishes every rank's updated slice.

On a GPU mesh (p > 1) both arenas are ``memAlloc`` tensors: mapped into every peer once, so the
reduce-scatter and the all-gather run the zero-copy IPC kernels (bench/collectives.py config 3:
4 GB bf16 in 7.0 ms at 8 ranks, profiles/r3/config3/).  ``close()`` frees them.
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional

import torch

from ..operands import Operand, Operands
from ..operators import Operators, dtype_of_torch, for_dtype

_OPERAND = {torch.float32: Operands.FLOAT_OPERAND, torch.float64: Operands.DOUBLE_OPERAND,
            torch.bfloat16: Operands.BF16_OPERAND, torch.float16: Operands.HALF_OPERAND}


class _Group:
    """The parameters of one dtype: arenas, this rank's slice, its master copy."""

    def __init__(self, params: List[torch.nn.Parameter], p: int, r: int, comm, memalloc: bool,
                 master_dtype: torch.dtype):
        dt = params[0].dtype
        self.params = params
        self.dtype = dt
        self.operand: Operand = _OPERAND[dt]()
        self.op = for_dtype(Operators.Float.SUM, dtype_of_torch(dt))
        es = params[0].element_size()
        unit = p * max(1, 16 // es)                       # every slice a whole number of 16-byte vectors
        self.numel = sum(q.numel() for q in params)
        self.n = -(-self.numel // unit) * unit
        self.shard = self.n // p
        self.lo, self.hi = r * self.shard, (r + 1) * self.shard
        dev = params[0].device
        alloc = (lambda: comm.memAlloc(self.n, dt, device=dev)) if memalloc else \
            (lambda: torch.empty(self.n, dtype=dt, device=dev))
        self.param_arena = alloc()
        self.grad_arena = alloc()
        self.param_arena.zero_()
        self.grad_arena.zero_()
        off = 0
        with torch.no_grad():
            for q in params:
                v = self.param_arena[off:off + q.numel()].view_as(q)
                v.copy_(q)
                q.data = v                                # the module now computes from the arena
                q.grad = self.grad_arena[off:off + q.numel()].view_as(q)
                off += q.numel()
        mine = self.param_arena[self.lo:self.hi]
        self.aliased = dt == master_dtype or dt in (torch.float32, torch.float64)
        if self.aliased:
            self.master = torch.nn.Parameter(mine)        # shares the arena's storage: stepped in place
        else:
            self.master = torch.nn.Parameter(mine.detach().to(master_dtype).clone())


class ZeroOptimizer:
    """Sharded-optimizer wrapper.  ``ZeroOptimizer(comm, model.parameters(), torch.optim.AdamW,
    lr=1e-3)``; per step: ``zero_grad()``, forward/backward, ``step()``.  All ranks must build it
    with the same parameter list (the constructor is collective when it allocates memAlloc
    arenas)."""

    def __init__(self, comm, params: Iterable[torch.nn.Parameter], optimizer=torch.optim.AdamW,
                 average: bool = True, max_grad_norm: Optional[float] = None,
                 master_dtype: torch.dtype = torch.float32, **optim_kwargs):
        self.comm = comm
        self.p, self.r = comm.getSlaveNum(), comm.getRank()
        self.average = average
        self.max_grad_norm = max_grad_norm
        params = [q for q in params if q.requires_grad]
        if not params:
            raise ValueError("no trainable parameters")
        by_dtype: Dict[torch.dtype, List[torch.nn.Parameter]] = {}
        for q in params:                                 # registration order: identical on every rank
            if q.dtype not in _OPERAND:
                raise ValueError(f"ZeroOptimizer: unsupported parameter dtype {q.dtype}")
            by_dtype.setdefault(q.dtype, []).append(q)
        self.cuda = params[0].is_cuda
        self._memalloc = self.cuda and self.p > 1 and hasattr(comm, "memAlloc")
        self.groups = [_Group(g, self.p, self.r, comm, self._memalloc, master_dtype) for g in by_dtype.values()]
        self.optim = optimizer([g.master for g in self.groups], **optim_kwargs)
        self._last_norm: Optional[torch.Tensor] = None

    # ------------------------------------------------------------------ step
    def zero_grad(self) -> None:
        for g in self.groups:
            g.grad_arena.zero_()

    def _reduce_scatter(self) -> None:
        for g in self.groups:
            if self.p > 1:
                self.comm.reduceScatterArray(g.grad_arena, g.operand, g.op, 0, [g.shard] * self.p)
            sl = g.grad_arena[g.lo:g.hi]
            if g.aliased:
                g.master.grad = sl                        # the slice itself: averaged in place below
            else:
                g.master.grad = sl.to(g.master.dtype)
            if self.average and self.p > 1:
                g.master.grad.mul_(1.0 / self.p)

    def _clip(self) -> None:
        """Global-norm clipping over the sharded gradient: each rank's slice square-sum, one
        1-element SUM allreduce, the coefficient applied on the device (no host sync)."""
        dev = self.groups[0].master.device
        sq = torch.zeros(1, dtype=torch.float64 if not self.cuda else torch.float32, device=dev)
        for g in self.groups:
            sq += g.master.grad.double().square().sum() if not self.cuda else g.master.grad.float().square().sum()
        if self.p > 1:
            opnd = Operands.DOUBLE_OPERAND() if sq.dtype == torch.float64 else Operands.FLOAT_OPERAND()
            op = Operators.Double.SUM if sq.dtype == torch.float64 else Operators.Float.SUM
            self.comm.allreduceArray(sq, opnd, op, 0, 1)
        norm = sq.sqrt()
        coef = torch.clamp(self.max_grad_norm / (norm + 1e-6), max=1.0)
        for g in self.groups:
            g.master.grad.mul_(coef.to(g.master.grad.dtype))
        self._last_norm = norm

    def _all_gather(self) -> None:
        for g in self.groups:
            if not g.aliased:
                with torch.no_grad():
                    g.param_arena[g.lo:g.hi].copy_(g.master)
            if self.p > 1:
                froms = [i * g.shard for i in range(self.p)]
                tos = [(i + 1) * g.shard for i in range(self.p)]
                self.comm.allgatherArray(g.param_arena, g.operand, froms, tos)

    def step(self) -> None:
        """Collective: reduce-scatter the gradients, step this rank's slice, all-gather the
        parameters."""
        self._reduce_scatter()
        if self.max_grad_norm is not None:
            self._clip()
        self.optim.step()
        self._all_gather()

    @property
    def grad_norm(self) -> Optional[float]:
        """The pre-clip global gradient norm of the last step (when clipping is on)."""
        return None if self._last_norm is None else float(self._last_norm)

    # ------------------------------------------------------------------ state
    def state_dict(self) -> dict:
        """This rank's shard: the inner optimizer's state and the master slices (a sharded
        checkpoint — every rank saves its own; ``load_state_dict`` needs the same p and rank)."""
        return {"p": self.p, "rank": self.r, "optim": self.optim.state_dict(),
                "masters": [g.master.detach().cpu().clone() for g in self.groups]}

    def load_state_dict(self, sd: dict) -> None:
        if sd["p"] != self.p or sd["rank"] != self.r:
            raise ValueError(f"shard checkpoint is for rank {sd['rank']}/{sd['p']}, this is {self.r}/{self.p}")
        with torch.no_grad():
            for g, m in zip(self.groups, sd["masters"]):
                g.master.copy_(m)
        self.optim.load_state_dict(sd["optim"])
        self._all_gather()                                # every rank's parameters from the restored slices

    def close(self) -> None:
        """Collective: drop the parameters' ``.grad`` views and free the memAlloc arenas.  The
        parameters keep their values (copied out of the arena first)."""
        for g in self.groups:
            with torch.no_grad():
                for q in g.params:
                    q.data = q.data.clone()
                    q.grad = None
            if self._memalloc:
                self.comm.memFree(g.param_arena)
                self.comm.memFree(g.grad_arena)
        self.groups = []


def train_zero(comm, steps: int = 5, global_batch: int = 64, din: int = 64, hidden: int = 128, dout: int = 16,
               lr: float = 0.01, device="cpu", dtype=torch.float32, max_grad_norm=None) -> List[float]:
    """The MLP of :mod:`mp4x.models.mlp` trained data-parallel with AdamW under ZeroOptimizer;
    returns the GLOBAL loss per step."""
    from .mlp import MLP, synthetic_batch
    p, r = comm.getSlaveNum(), comm.getRank()
    torch.manual_seed(0)
    model = MLP(din, hidden, dout).to(device=device, dtype=dtype)
    opt = ZeroOptimizer(comm, model.parameters(), torch.optim.AdamW, lr=lr, weight_decay=0.01,
                        max_grad_norm=max_grad_norm)
    losses = []
    shard = global_batch // p
    for step in range(steps):
        x, y = synthetic_batch(step, global_batch, din, dout, device)
        xs, ys = x[r * shard:(r + 1) * shard].to(dtype), y[r * shard:(r + 1) * shard].to(dtype)
        opt.zero_grad()
        loss = torch.nn.functional.mse_loss(model(xs), ys)
        loss.backward()
        opt.step()
        lv = float(loss.detach().float().cpu())
        losses.append(comm.allreduce(lv, Operands.DOUBLE_OPERAND(), Operators.Double.SUM) / p if p > 1 else lv)
    opt.close()
    return losses


def train_single_adamw(steps: int = 5, global_batch: int = 64, din: int = 64, hidden: int = 128, dout: int = 16,
                       lr: float = 0.01, device="cpu", dtype=torch.float32, max_grad_norm=None) -> List[float]:
    from .mlp import MLP, synthetic_batch
    torch.manual_seed(0)
    model = MLP(din, hidden, dout).to(device=device, dtype=dtype)
    opt = torch.optim.AdamW(model.parameters(), lr=lr, weight_decay=0.01)
    losses = []
    for step in range(steps):
        x, y = synthetic_batch(step, global_batch, din, dout, device)
        opt.zero_grad()
        loss = torch.nn.functional.mse_loss(model(x.to(dtype)), y.to(dtype))
        loss.backward()
        if max_grad_norm is not None:
            torch.nn.utils.clip_grad_norm_(model.parameters(), max_grad_norm)
        opt.step()
        losses.append(float(loss.detach().float().cpu()))
    return losses
