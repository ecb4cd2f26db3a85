"""Collective back-ends used by the device engine.

``TorchColl``    the production path: ``torch.distributed`` with the ``nccl`` backend, i.e.
                 RCCL over xGMI (gloo for CPU tensors in tests).
``LoopbackColl`` an in-process fake: p "virtual ranks" are threads of ONE process that share
                 a hub; every collective is computed from the ranks' published tensors.  It
                 lets the whole device engine (two-shot a2a schedule, fp8 / bf16 codecs,
                 sparse map exchange, p2p gather/scatter) run with real HIP kernels on a
                 single GPU — RCCL refuses two ranks on one device — and without any GPU on
                 CPU tensors (the "fake backend" SURVEY §4 asks for).
"""
from __future__ import annotations

import threading
from collections import defaultdict
from typing import List, Sequence, Tuple

import torch
import torch.distributed as dist

from ..operators import OpCode

_RCCL_OPS = {OpCode.SUM: dist.ReduceOp.SUM, OpCode.MAX: dist.ReduceOp.MAX,
             OpCode.MIN: dist.ReduceOp.MIN, OpCode.PROD: dist.ReduceOp.PRODUCT}


# dtypes the transports move natively; anything else (int16, ...) moves as its bytes in the
# data-movement collectives (RCCL and gloo have no int16 type; a copy is a copy)
_MOVE_DTYPES = {torch.float64, torch.float32, torch.bfloat16, torch.float16, torch.int64, torch.int32,
                torch.int8, torch.uint8}


def _mv(t: torch.Tensor) -> torch.Tensor:
    return t if t.dtype in _MOVE_DTYPES else t.view(torch.uint8)


def _scale(splits, t: torch.Tensor):
    """all_to_all splits of ``t`` as moved by :func:`_mv`: the uint8 view widens only the LAST
    dimension, so dim-0 splits grow by the element size for 1-D tensors only (an [n, dim] int16
    tensor keeps its row splits)."""
    if splits is None or t.dtype in _MOVE_DTYPES or t.dim() > 1:
        return splits
    return [x * t.element_size() for x in splits]


class TorchColl:
    """``order``: the owning engine's stream-order guard (parallel/order.py).  RCCL orders a
    communicator's collectives on its own stream after the CURRENT stream of each call; the guard
    first joins the current stream to the stream of the communicator's previous launch (an IPC
    kernel, or an RCCL call issued from another stream), so IPC and RCCL calls share one order."""
    order = None

    def __init__(self, pg, backend: str):
        self.pg = pg
        self.backend = backend
        self.gather_into_tensor_ok = backend != "gloo"
        self.reduce_scatter_ok = backend != "gloo"

    def _enter(self, t) -> None:
        o = self.order
        if o is not None and getattr(t, "is_cuda", False):
            from ..ops.native import stream_ptr
            o.enter(stream_ptr())

    def all_reduce(self, t, code, avg: bool = False):
        """``avg``: SUM then divide by the group size inside the collective (ncclAvg)."""
        self._enter(t)
        dist.all_reduce(t, op=dist.ReduceOp.AVG if avg else _RCCL_OPS[code], group=self.pg)

    def reduce(self, t, dst, code):
        self._enter(t)
        dist.reduce(t, dst=dst, op=_RCCL_OPS[code], group=self.pg)

    def broadcast(self, t, src):
        self._enter(t)
        dist.broadcast(_mv(t), src=src, group=self.pg)

    def all_to_all_single(self, out, inp, out_splits=None, in_splits=None):
        self._enter(out)
        dist.all_to_all_single(_mv(out), _mv(inp), _scale(out_splits, out), _scale(in_splits, inp), group=self.pg)

    def all_gather_into_tensor(self, out, inp):
        self._enter(out)
        dist.all_gather_into_tensor(_mv(out), _mv(inp), group=self.pg)

    def all_gather(self, outs, t):
        self._enter(t)
        dist.all_gather([_mv(o) for o in outs], _mv(t), group=self.pg)

    def reduce_scatter_tensor(self, out, inp, code):
        self._enter(out)
        dist.reduce_scatter_tensor(out, inp, op=_RCCL_OPS[code], group=self.pg)

    def p2p(self, sends: Sequence[Tuple[torch.Tensor, int]], recvs: Sequence[Tuple[torch.Tensor, int]]):
        ops = [dist.P2POp(dist.isend, _mv(t), j, group=self.pg) for t, j in sends]
        ops += [dist.P2POp(dist.irecv, _mv(t), j, group=self.pg) for t, j in recvs]
        # gloo's send/recv of a DEVICE tensor is not ordered after the kernels queued on the
        # current stream (one-GPU rehearsals stand gloo in for RCCL): drain the stream first.
        # RCCL orders its own stream after the current one, so the production path never waits.
        gloo_dev = self.backend == "gloo" and any(t.is_cuda for t, _ in list(sends) + list(recvs))
        if ops:
            self._enter((list(sends) + list(recvs))[0][0])
            if gloo_dev:
                torch.cuda.current_stream().synchronize()
            for w in dist.batch_isend_irecv(ops):
                w.wait()
            if gloo_dev:
                torch.cuda.current_stream().synchronize()

    def barrier(self):
        dist.barrier(group=self.pg)


class LoopbackHub:
    """Shared state of p virtual ranks living in one process."""

    def __init__(self, p: int):
        self.p = p
        self.bar = threading.Barrier(p)
        self.slots: List[object] = [None] * p
        self.box = {}
        self.cv = threading.Condition()

    def coll(self, rank: int) -> "LoopbackColl":
        return LoopbackColl(self, rank)


def _combine(code, a, b):
    if code == OpCode.SUM:
        return a + b
    if code == OpCode.MAX:
        return torch.maximum(a, b)
    if code == OpCode.MIN:
        return torch.minimum(a, b)
    if code == OpCode.PROD:
        return a * b
    raise ValueError(code)


class LoopbackColl:
    gather_into_tensor_ok = True
    reduce_scatter_ok = True
    backend = "loopback"

    def __init__(self, hub: LoopbackHub, rank: int):
        self.hub = hub
        self.rank = rank
        self.p = hub.p
        self._seq = defaultdict(int)

    def _sync(self, t=None):
        if (t is not None and t.is_cuda) or torch.cuda.is_available():
            torch.cuda.synchronize()

    def _exchange(self, obj):
        """Publish obj, return every rank's object (after all published)."""
        self._sync()
        self.hub.slots[self.rank] = obj
        self.hub.bar.wait()
        out = list(self.hub.slots)
        self.hub.bar.wait()
        return out

    def _exchange_apply(self, obj, fn):
        """Publish obj, run ``fn(every rank's obj)`` while all of them are still published (the
        closing barrier keeps every peer's tensor alive and unmodified until everyone has
        copied from it): the data-movement collectives read peers' tensors directly instead of
        publishing clones."""
        self._sync()
        self.hub.slots[self.rank] = obj
        self.hub.bar.wait()
        try:
            fn(list(self.hub.slots))
            self._sync()
        finally:
            self.hub.bar.wait()

    def all_reduce(self, t, code, avg: bool = False):
        xs = self._exchange(t.clone())
        acc = xs[0].clone()
        for x in xs[1:]:
            acc = _combine(code, acc, x)
        if avg:
            acc = acc / self.p
        t.copy_(acc)
        self._sync()

    def reduce(self, t, dst, code):
        xs = self._exchange(t.clone())
        if self.rank == dst:
            acc = xs[0].clone()
            for x in xs[1:]:
                acc = _combine(code, acc, x)
            t.copy_(acc)
        self._sync()

    def broadcast(self, t, src):
        xs = self._exchange(t.clone() if self.rank == src else None)
        if self.rank != src:
            t.copy_(xs[src])
        self._sync()

    def all_to_all_single(self, out, inp, out_splits=None, in_splits=None):
        p = self.p
        if in_splits is None:
            in_splits = [inp.shape[0] // p] * p
        offs = [0]
        for s in in_splits:
            offs.append(offs[-1] + s)
        r = self.rank

        def take(slots):
            o = 0
            for src, so in slots:
                g = src[so[r]:so[r + 1]]
                out[o:o + g.shape[0]].copy_(g)
                o += g.shape[0]
        self._exchange_apply((inp, offs), take)

    def all_gather_into_tensor(self, out, inp):
        flat = out.view(-1)
        n = inp.numel()

        def take(xs):
            for j, x in enumerate(xs):
                flat[j * n:(j + 1) * n].copy_(x.reshape(-1))
        self._exchange_apply(inp, take)

    def all_gather(self, outs, t):
        def take(xs):
            for o, x in zip(outs, xs):
                o.copy_(x)
        self._exchange_apply(t, take)

    def reduce_scatter_tensor(self, out, inp, code):
        xs = self._exchange(inp.clone())
        n = out.numel()
        acc = xs[0][self.rank * n:(self.rank + 1) * n].clone()
        for x in xs[1:]:
            acc = _combine(code, acc, x[self.rank * n:(self.rank + 1) * n])
        out.copy_(acc.view_as(out))
        self._sync()

    def p2p(self, sends, recvs):
        self._sync()
        with self.hub.cv:
            for t, j in sends:
                k = (self.rank, j, self._seq[("s", j)])
                self._seq[("s", j)] += 1
                self.hub.box[k] = t.clone()
            self.hub.cv.notify_all()
        for t, j in recvs:
            k = (j, self.rank, self._seq[("r", j)])
            self._seq[("r", j)] += 1
            with self.hub.cv:
                while k not in self.hub.box:
                    self.hub.cv.wait(1.0)
                v = self.hub.box.pop(k)
            t.copy_(v)
        self._sync()

    def barrier(self):
        self.hub.bar.wait()


class _FakeComm:
    """Minimal communicator facade for a loopback virtual rank."""

    def __init__(self, rank: int, p: int):
        self.rank = rank
        self.slaveNum = p
        self.server = None
        self.transport = None


def loopback_engines(p: int, device=None):
    """p DeviceEngines sharing one LoopbackHub (drive each from its own thread)."""
    from .device_engine import DeviceEngine
    hub = LoopbackHub(p)
    return [DeviceEngine(_FakeComm(r, p), coll=hub.coll(r), device=device) for r in range(p)]
