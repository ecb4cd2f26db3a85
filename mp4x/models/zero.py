"""ZeRO-style sharded optimizer: BASELINE config 3's reduceScatter + allgather pattern inside a
training loop (the reference has no optimizer; its ``reduceScatterArray`` / ``allgatherArray``,
ProcessCommSlave.java:1174 / :620, are the collectives this is built from).

Every trainable parameter lives in a flat per-dtype arena (``param.data`` is a view) and its
gradient in a second arena (``param.grad`` is a view; autograd accumulates into it in place).
Parameters are grouped into buckets (reverse registration order ~ backward order, ``bucket_mb``
each); every bucket is padded to a multiple of ``p`` 16-byte vectors, so rank ``r`` owns the
contiguous, 16-byte-aligned r-th slice of every bucket.  A step is:

1. ``reduceScatterArray`` of each bucket's gradients — rank r ends up with the reduced gradient
   of its slices only (1/p of the bytes of an allreduce on every link).  With ``overlap`` (the
   default on GPUs) a bucket's reduce-scatter is launched on a side HIP stream by the autograd
   hook of its last gradient, so it overlaps the rest of the backward pass (ZeRO-2);
2. the 1/p average and optional global-norm clipping on the slices (the norm is one 1-element
   allreduce; the clip coefficient stays on the device, no host sync);
3. the inner optimizer (any ``torch.optim`` class; elementwise ones such as AdamW / SGD give the
   same trajectory as unsharded training) steps the slices' master copies — fp32 for bf16 /
   fp16 parameters, aliases of the slices themselves for fp32 / fp64 — so optimizer state is
   1/p per rank;
4. ``allgatherArray`` of each bucket's parameters publishes every rank's updated slice.

Gradient accumulation over several backward passes: run all but the last inside
``with opt.no_sync():`` (the hooks then launch nothing; ``step()`` reduces every bucket).

On a GPU mesh (p > 1) both arenas are ``memAlloc`` tensors: mapped into every peer once, so the
reduce-scatters and all-gathers of every bucket (views of the arenas) run the zero-copy IPC
kernels (bench/collectives.py config 3: 4 GB bf16 in 7.0 ms at 8 ranks, profiles/r3/config3/).
``close()`` frees them.
"""
from __future__ import annotations

import contextlib
import os
from typing import Dict, Iterable, List, Optional

import torch

from ..operands import Operand, Operands
from ..operators import Operators, dtype_of_torch, for_dtype

_OPERAND = {torch.float32: Operands.FLOAT_OPERAND, torch.float64: Operands.DOUBLE_OPERAND,
            torch.bfloat16: Operands.BF16_OPERAND, torch.float16: Operands.HALF_OPERAND}


def _padded(params: List[torch.nn.Parameter], p: int) -> int:
    unit = p * max(1, 16 // params[0].element_size())     # every slice whole 16-byte vectors
    return -(-sum(q.numel() for q in params) // unit) * unit


class _Bucket:
    """A run of same-dtype parameters: its windows of the two arenas, this rank's slice, the
    slice's master copy, and the backward-hook bookkeeping."""

    def __init__(self, params: List[torch.nn.Parameter], p: int, r: int, param_arena: torch.Tensor,
                 grad_arena: torch.Tensor, off: int, master_dtype: torch.dtype):
        dt = params[0].dtype
        self.params = params
        self.operand: Operand = _OPERAND[dt]()
        self.op = for_dtype(Operators.Float.SUM, dtype_of_torch(dt))
        self.n = _padded(params, p)
        self.shard = self.n // p
        self.lo, self.hi = r * self.shard, (r + 1) * self.shard      # within the bucket
        self.param = param_arena[off:off + self.n]
        self.grad = grad_arena[off:off + self.n]
        o = 0
        with torch.no_grad():
            for q in params:
                v = self.param[o:o + q.numel()].view_as(q)
                v.copy_(q)
                q.data = v                                # the module now computes from the arena
                q.grad = self.grad[o:o + q.numel()].view_as(q)
                o += q.numel()
        mine = self.param[self.lo:self.hi]
        self.aliased = dt == master_dtype or dt in (torch.float32, torch.float64)
        if self.aliased:
            self.master = torch.nn.Parameter(mine)        # shares the arena's storage: stepped in place
        else:
            self.master = torch.nn.Parameter(mine.detach().to(master_dtype).clone())
        self.pending = len(params)
        self.launched = False


class ZeroOptimizer:
    """Sharded-optimizer wrapper.  ``ZeroOptimizer(comm, model.parameters(), torch.optim.AdamW,
    lr=1e-3)``; per step: ``zero_grad()``, forward/backward, ``step()``.  All ranks must build it
    with the same parameter list (the constructor is collective when it allocates memAlloc
    arenas).  ``bucket_mb``: reduce-scatter granularity (default ``MP4X_BUCKET_MB`` = 64);
    ``overlap``: launch each bucket's reduce-scatter from the backward hooks (default: on GPUs)."""

    def __init__(self, comm, params: Iterable[torch.nn.Parameter], optimizer=torch.optim.AdamW,
                 average: bool = True, max_grad_norm: Optional[float] = None,
                 master_dtype: torch.dtype = torch.float32, bucket_mb: Optional[float] = None,
                 overlap: Optional[bool] = None, **optim_kwargs):
        self.comm = comm
        self.p, self.r = comm.getSlaveNum(), comm.getRank()
        self.average = average
        self.max_grad_norm = max_grad_norm
        params = [q for q in params if q.requires_grad]
        if not params:
            raise ValueError("no trainable parameters")
        for q in params:
            if q.dtype not in _OPERAND:
                raise ValueError(f"ZeroOptimizer: unsupported parameter dtype {q.dtype}")
        cap = int((bucket_mb or float(os.environ.get("MP4X_BUCKET_MB", 64))) * (1 << 20))
        runs: Dict[torch.dtype, List[List[torch.nn.Parameter]]] = {}
        for q in reversed(params):                       # backward order; identical on every rank
            rs = runs.setdefault(q.dtype, [[]])
            if rs[-1] and (sum(x.numel() for x in rs[-1]) + q.numel()) * q.element_size() > cap:
                rs.append([])
            rs[-1].append(q)
        self.cuda = params[0].is_cuda
        self.overlap = (self.cuda if overlap is None else overlap) and self.p > 1
        self._memalloc = self.cuda and self.p > 1 and hasattr(comm, "memAlloc")
        self.buckets: List[_Bucket] = []
        self._arenas: List[torch.Tensor] = []
        for dt, rs in runs.items():                      # dtype order of first appearance: agreed
            total = sum(_padded(b, self.p) for b in rs)
            dev = rs[0][0].device
            pa, ga = ((comm.memAlloc(total, dt, device=dev), comm.memAlloc(total, dt, device=dev))
                      if self._memalloc else
                      (torch.empty(total, dtype=dt, device=dev), torch.empty(total, dtype=dt, device=dev)))
            pa.zero_()
            ga.zero_()
            self._arenas += [pa, ga]
            off = 0
            for b in rs:
                self.buckets.append(_Bucket(b, self.p, self.r, pa, ga, off, master_dtype))
                off += self.buckets[-1].n
        self._owner = {}
        self._hooks = []
        for b in self.buckets:
            for q in b.params:
                self._owner[q] = b
                if self.overlap:
                    self._hooks.append(q.register_post_accumulate_grad_hook(self._hook))
        self.stream = torch.cuda.Stream() if self.cuda and self.overlap else None
        self._sync_grads = True
        self.optim = optimizer([b.master for b in self.buckets], **optim_kwargs)
        self._last_norm: Optional[torch.Tensor] = None

    # ------------------------------------------------------------------ reduce-scatter
    def _hook(self, q) -> None:
        b = self._owner[q]
        b.pending -= 1
        if b.pending == 0 and self._sync_grads:
            self._launch(b)

    def _launch(self, b: _Bucket) -> None:
        b.launched = True
        if self.p == 1:
            return
        if self.stream is not None:
            ev = torch.cuda.Event()
            ev.record()                                  # the bucket's gradients are complete here
            with torch.cuda.stream(self.stream):
                self.stream.wait_event(ev)
                self.comm.reduceScatterArray(b.grad, b.operand, b.op, 0, [b.shard] * self.p)
        else:
            self.comm.reduceScatterArray(b.grad, b.operand, b.op, 0, [b.shard] * self.p)

    @contextlib.contextmanager
    def no_sync(self):
        """Backward passes inside accumulate gradients locally (no reduce-scatter launched)."""
        self._sync_grads = False
        try:
            yield
        finally:
            self._sync_grads = True
            for b in self.buckets:
                b.pending = len(b.params)

    def _reduce_scatter(self) -> None:
        for b in self.buckets:                           # buckets no hook launched (unused params, no overlap)
            if not b.launched:
                self._launch(b)
        if self.stream is not None:
            torch.cuda.current_stream().wait_stream(self.stream)
        for b in self.buckets:
            sl = b.grad[b.lo:b.hi]
            b.master.grad = sl if b.aliased else sl.to(b.master.dtype)   # aliased: averaged in place
            if self.average and self.p > 1:
                b.master.grad.mul_(1.0 / self.p)
            b.pending = len(b.params)
            b.launched = False

    def _clip(self) -> None:
        """Global-norm clipping over the sharded gradient: each rank's slice square-sum, one
        1-element SUM allreduce, the coefficient applied on the device (no host sync)."""
        dev = self.buckets[0].master.device
        acc = torch.float32 if self.cuda else torch.float64
        sq = torch.zeros(1, dtype=acc, device=dev)
        for b in self.buckets:
            sq += b.master.grad.to(acc).square().sum()
        if self.p > 1:
            if acc == torch.float64:
                self.comm.allreduceArray(sq, Operands.DOUBLE_OPERAND(), Operators.Double.SUM, 0, 1)
            else:
                self.comm.allreduceArray(sq, Operands.FLOAT_OPERAND(), Operators.Float.SUM, 0, 1)
        norm = sq.sqrt()
        coef = torch.clamp(self.max_grad_norm / (norm + 1e-6), max=1.0)
        for b in self.buckets:
            b.master.grad.mul_(coef.to(b.master.grad.dtype))
        self._last_norm = norm

    def _all_gather(self) -> None:
        for b in self.buckets:
            if not b.aliased:
                with torch.no_grad():
                    b.param[b.lo:b.hi].copy_(b.master)
            if self.p > 1:
                froms = [i * b.shard for i in range(self.p)]
                tos = [(i + 1) * b.shard for i in range(self.p)]
                self.comm.allgatherArray(b.param, b.operand, froms, tos)

    # ------------------------------------------------------------------ public
    def zero_grad(self) -> None:
        for a in self._arenas[1::2]:
            a.zero_()

    def step(self) -> None:
        """Collective: reduce-scatter the gradients (what the backward hooks did not launch yet),
        step this rank's slices, all-gather the parameters."""
        self._reduce_scatter()
        if self.max_grad_norm is not None:
            self._clip()
        self.optim.step()
        self._all_gather()

    @property
    def grad_norm(self) -> Optional[float]:
        """The pre-clip global gradient norm of the last step (when clipping is on)."""
        return None if self._last_norm is None else float(self._last_norm)

    def state_dict(self) -> dict:
        """This rank's shard: the inner optimizer's state and the master slices (a sharded
        checkpoint — every rank saves its own; ``load_state_dict`` needs the same p and rank)."""
        return {"p": self.p, "rank": self.r, "optim": self.optim.state_dict(),
                "masters": [b.master.detach().cpu().clone() for b in self.buckets]}

    def load_state_dict(self, sd: dict) -> None:
        if sd["p"] != self.p or sd["rank"] != self.r:
            raise ValueError(f"shard checkpoint is for rank {sd['rank']}/{sd['p']}, this is {self.r}/{self.p}")
        if len(sd["masters"]) != len(self.buckets):
            raise ValueError("shard checkpoint has a different bucket layout")
        with torch.no_grad():
            for b, m in zip(self.buckets, sd["masters"]):
                b.master.copy_(m)
        self.optim.load_state_dict(sd["optim"])
        self._all_gather()                                # every rank's parameters from the restored slices

    def close(self) -> None:
        """Collective: drop the hooks and the parameters' ``.grad`` views and free the memAlloc
        arenas.  The parameters keep their values (copied out of the arena first)."""
        if self.stream is not None:
            torch.cuda.current_stream().wait_stream(self.stream)
        for h in self._hooks:
            h.remove()
        self._hooks = []
        for b in self.buckets:
            with torch.no_grad():
                for q in b.params:
                    q.data = q.data.clone()
                    q.grad = None
        self.buckets = []
        self._owner = {}
        if self._memalloc:
            for a in self._arenas:
                self.comm.memFree(a)
        self._arenas = []


def train_zero(comm, steps: int = 5, global_batch: int = 64, din: int = 64, hidden: int = 128, dout: int = 16,
               lr: float = 0.01, device="cpu", dtype=torch.float32, max_grad_norm=None,
               bucket_mb: Optional[float] = None, overlap: Optional[bool] = None, micro: int = 1) -> List[float]:
    """The MLP of :mod:`mp4x.models.mlp` trained data-parallel with AdamW under ZeroOptimizer
    (``micro`` gradient-accumulation micro-batches per step); returns the GLOBAL loss per step."""
    from .mlp import MLP, synthetic_batch
    p, r = comm.getSlaveNum(), comm.getRank()
    torch.manual_seed(0)
    model = MLP(din, hidden, dout).to(device=device, dtype=dtype)
    opt = ZeroOptimizer(comm, model.parameters(), torch.optim.AdamW, lr=lr, weight_decay=0.01,
                        max_grad_norm=max_grad_norm, bucket_mb=bucket_mb, overlap=overlap)
    losses = []
    shard = global_batch // p
    mb = shard // micro
    for step in range(steps):
        x, y = synthetic_batch(step, global_batch, din, dout, device)
        xs, ys = x[r * shard:(r + 1) * shard].to(dtype), y[r * shard:(r + 1) * shard].to(dtype)
        opt.zero_grad()
        tot = 0.0
        for i in range(micro):
            ctx = opt.no_sync() if i < micro - 1 else contextlib.nullcontext()
            with ctx:
                loss = torch.nn.functional.mse_loss(model(xs[i * mb:(i + 1) * mb]), ys[i * mb:(i + 1) * mb]) / micro
                loss.backward()
            tot += float(loss.detach().float().cpu())
        opt.step()
        losses.append(comm.allreduce(tot, Operands.DOUBLE_OPERAND(), Operators.Double.SUM) / p if p > 1 else tot)
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
