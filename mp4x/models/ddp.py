"""Data-parallel gradient synchronisation on top of ProcessComm (the reference's raison
d'être: ytk-learn syncs L-BFGS / GBDT statistics with ``allreduceArray``, README.md:268-280).

``GradientSynchronizer`` buckets parameters (reverse registration order ≈ backward order)
into flat buffers, makes every ``param.grad`` a VIEW into its bucket (no flatten/unflatten
copies), and launches each bucket's allreduce as soon as the last gradient of the bucket
has been accumulated — on a dedicated HIP stream, so RCCL / the IPC kernels overlap the
rest of the backward pass.  The 1/p average is fused into the allreduce itself (the IPC
kernels scale the reduced value before their final store, RCCL uses ncclAvg, the fp8 path
scales before re-quantising), so no separate pass over the buckets runs; ``finish()`` only
joins the streams.  Buckets are views of one ``memAlloc`` arena per dtype (mapped into every
peer at any size), so the two-shot runs zero-copy on them; ``close()`` frees it.

Bucket size: xGMI is point-to-point (7 links x ~153 GB/s per MI355X) and RCCL splits a
message over channels/links; buckets of 32-128 MiB keep every link busy while leaving
enough buckets to overlap with backward.  Default 64 MiB (``MP4X_BUCKET_MB``).
"""
from __future__ import annotations

import os
from typing import Iterable, List, Optional

import torch

from ..operands import Operands
from ..operators import Operators, for_dtype, dtype_of_torch


class _Bucket:
    def __init__(self, params: List[torch.nn.Parameter], buffer: torch.Tensor):
        self.params = params
        self.buffer = buffer
        self.pending = len(params)
        self.event = None
        self.averaged = False
        off = 0
        self.views = []
        for p in params:
            v = self.buffer[off:off + p.numel()].view_as(p)
            self.views.append(v)
            off += p.numel()


class GradientSynchronizer:
    def __init__(self, comm, params: Iterable[torch.nn.Parameter], bucket_mb: Optional[float] = None,
                 average: bool = True, codec: Optional[str] = None, autotune: bool = False):
        self.comm = comm
        self.p = comm.getSlaveNum()
        self.average = average
        self.operand = Operands.FLOAT_OPERAND(codec=codec)
        params = [p for p in params if p.requires_grad]
        if not params:
            raise ValueError("no trainable parameters")
        cap = int((bucket_mb or float(os.environ.get("MP4X_BUCKET_MB", 64))) * (1 << 20))
        groups: List[List[torch.nn.Parameter]] = []
        cur: List[torch.nn.Parameter] = []
        size = 0
        for p in reversed(params):
            if cur and (size + p.numel() * p.element_size() > cap or p.dtype != cur[0].dtype):
                groups.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += p.numel() * p.element_size()
        if cur:
            groups.append(cur)
        self.cuda = groups[0][0].is_cuda
        # One arena per dtype holds every bucket of that dtype, 16-byte aligned bucket offsets.
        # On a GPU mesh it is a memAlloc tensor: mapped into every peer once, at any size, so
        # every bucket's allreduce runs the zero-copy kernels (no caching-allocator segment that
        # might be too large to map, no registration to forget).
        self._arenas: List[torch.Tensor] = []
        self._memalloc = self.cuda and self.p > 1 and hasattr(self.comm, "memAlloc")
        sizes, offs, totals = [], [], {}
        for g in groups:                                  # bucket offsets inside its dtype's arena
            es = g[0].element_size()
            align = max(1, 16 // es)
            n = -(-sum(p.numel() for p in g) // align) * align
            sizes.append(n)
            offs.append(totals.get(g[0].dtype, 0))
            totals[g[0].dtype] = offs[-1] + n
        arenas = {}
        for dt, total in totals.items():                  # same order on every rank: collective
            dev = next(g[0].device for g in groups if g[0].dtype == dt)
            if self._memalloc:
                arena = self.comm.memAlloc(total, dt, device=dev)
            else:
                arena = torch.empty(total, dtype=dt, device=dev)
            arena.zero_()
            arenas[dt] = arena
            self._arenas.append(arena)
        self.buckets: List[_Bucket] = [_Bucket(g, arenas[g[0].dtype][o:o + n])     # backward order
                                       for g, o, n in zip(groups, offs, sizes)]
        self._owner = {}
        for b in self.buckets:
            off = 0
            for p in b.params:
                p.grad = b.buffer[off:off + p.numel()].view_as(p)   # grads accumulate in the bucket
                off += p.numel()
                self._owner[p] = b
                p.register_post_accumulate_grad_hook(self._hook)
        self.stream = torch.cuda.Stream() if self.cuda else None
        self._launched: List[_Bucket] = []
        self.tuned = {}
        if autotune:
            self.autotune()

    def autotune(self):
        """Collective: measure the allreduce schedules once per distinct bucket (dtype, size
        class) and pin the fastest in the device engine (see ``DeviceEngine.autotune_allreduce``).
        Returns {bucket index: {algo: seconds}}."""
        if self.p == 1 or self.operand.codec:
            return self.tuned
        seen = set()
        for i, b in enumerate(self.buckets):
            key = (b.buffer.dtype, max(0, b.buffer.numel() * b.buffer.element_size() - 1).bit_length())
            if key in seen:
                continue
            seen.add(key)
            op = for_dtype(Operators.Float.SUM, dtype_of_torch(b.buffer.dtype))
            self.tuned[i] = self.comm.device.autotune_allreduce(b.buffer, op)
        return self.tuned

    def _hook(self, p):
        b = self._owner[p]
        b.pending -= 1
        if b.pending == 0:
            self._launch(b)

    def _launch(self, b: _Bucket):
        if self.p == 1:
            self._launched.append(b)
            return
        op = for_dtype(Operators.Float.SUM, dtype_of_torch(b.buffer.dtype))
        if self.cuda:
            ev = torch.cuda.Event()
            ev.record()                          # gradients of this bucket are complete on the compute stream
            with torch.cuda.stream(self.stream):
                self.stream.wait_event(ev)
                if self.average and b.buffer.is_floating_point() and hasattr(self.comm, "device"):
                    # average fused into the collective's final write (no extra HBM pass)
                    self.comm.device.allreduce(b.buffer, 0, b.buffer.numel(), op, self.operand, scale=1.0 / self.p)
                    b.averaged = True
                else:
                    self.comm.allreduceArray(b.buffer, self.operand, op, 0, b.buffer.numel())
        else:
            self.comm.allreduceArray(b.buffer, self.operand, op, 0, b.buffer.numel())
        self._launched.append(b)

    def finish(self):
        """Wait for every bucket, average, and re-arm for the next step."""
        for b in self.buckets:                   # buckets whose hooks did not fire (unused params)
            if b.pending > 0 and b not in self._launched:
                self._launch(b)
        if self.cuda:
            torch.cuda.current_stream().wait_stream(self.stream)
        if self.average and self.p > 1:
            for b in self.buckets:
                if not b.averaged:
                    b.buffer.mul_(1.0 / self.p)     # host buffers / integer buckets only
        for b in self.buckets:
            b.pending = len(b.params)
            b.averaged = False
        self._launched = []

    def zero_grad(self):
        for b in self.buckets:
            b.buffer.zero_()

    def close(self):
        """Collective: release the bucket arenas (``memFree``: the peers' mappings of them and
        the push scratch).  The parameters' ``.grad`` views are dropped first."""
        if self.cuda:
            torch.cuda.current_stream().wait_stream(self.stream)
        for b in self.buckets:
            for p in b.params:
                p.grad = None
        self.buckets = []
        self._owner = {}
        if self._memalloc:
            for a in self._arenas:
                self.comm.memFree(a)
        self._arenas = []
