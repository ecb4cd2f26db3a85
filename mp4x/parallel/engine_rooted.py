"""Rooted collectives of the device engine — broadcast, reduce, gather, scatter (mixin of
:class:`~mp4x.parallel.device_engine.DeviceEngine`; split out of device_engine.py in round 5).

Per call: a schedule pinned by the rooted autotuners, the zero-copy forms on a registered tensor,
the IPC copy plans / two-shot up to the direct tier, the piecewise IPC forms when no RCCL is
underneath, else RCCL (``ncclBroadcast`` / ``ncclReduce`` / grouped p2p).

Reference: broadcastArray = scatter + all-gather (ProcessCommSlave.java:750-775), reduceArray =
reduce-scatter + gather (:1390-1421), the binary-tree scatter (:1103-1159) and the dynamic-tree
gather (:440-520).
"""
from __future__ import annotations

import os

import torch

from ..ops.native import capturing_now
from ..utils.commutils import CommUtils


class RootedMixin:
    """broadcast / reduce / gather / scatter; state lives on the engine."""

    def broadcast(self, arr: torch.Tensor, frm: int, to: int, root: int, memo: bool = False):
        flat = self._flat(arr)
        if to > frm:
            t = self._root_tuned("broadcast", flat[frm:to], None)
            if t == "rccl":
                self._count("broadcast")
                self.coll.broadcast(flat[frm:to], root)
                return arr
            if t == "ipc" and self.ipc() is not None and self.ipc_large() is not None and \
                    self.ipc_large().broadcast_large(flat, frm, to, root):
                self._count("broadcast.ipc_large")
                return arr
            if (self.algo == "composite" or t == "composite") and to - frm >= self.p:
                # van de Geijn, the reference's schedule (ProcessCommSlave.java:750-775): scatter
                # from the root, then all-gather — kept for parity benchmarks (MP4X_DEVICE_ALGO)
                self._count("broadcast.composite")
                froms, tos, _ = CommUtils.even_split(frm, to, self.p)
                self.scatter(flat, froms, tos, root)
                self.allgather(flat, froms, tos)
                return arr
            if self.algo in ("", "auto") and self._zc_ok(flat) and self._zc_broadcast(flat, frm, to, root):
                self._count("broadcast.ipc_zc")
                return arr
            if self._ipc_small_ok(flat, (to - frm) * flat.element_size()) and \
                    self._plan_memo(memo, "broadcast", arr, (frm, to, root),
                                    lambda: self._ipc_obj.broadcast(flat, frm, to, root)):
                self._count("broadcast.ipc")
                return arr
            if self._dm_large_ok(flat) and self.ipc_large().broadcast_large(flat, frm, to, root):
                self._count("broadcast.ipc_large")
                return arr
            self._count("broadcast")
            self.coll.broadcast(flat[frm:to], root)
        return arr

    def _zc_broadcast(self, flat: torch.Tensor, frm: int, to: int, root: int) -> bool:
        """Broadcast on a registered tensor as the zero-copy all-gather whose only non-empty
        segment is the root's: every other rank pulls ``[frm, to)`` straight from the root's
        tensor over xGMI, one kernel at any size (no staging, no pieces).  False (nothing done,
        on every rank alike: ranges and registration are collective facts) otherwise."""
        if (to - frm) * flat.element_size() <= self.ipc_oneshot_max:
            return False                      # the latency tier keeps the one-kernel copy plan
        froms = [frm if j <= root else to for j in range(self.p)]
        tos = [frm if j < root else to for j in range(self.p)]
        return self._ipc_obj.allgather_registered(flat, froms, tos)

    def _dm_large_ok(self, flat: torch.Tensor) -> bool:
        """Piecewise IPC copy plans for broadcast / scatter / gather / all-gather above the
        direct tier.  ``MP4X_DM_LARGE``: ``auto`` (default) = when the transport is not RCCL
        (gloo standing in on GPU tensors moves device data through the host: 1-3 s per 80 MB in
        the one-GPU rehearsals), or when ``MP4X_DEVICE_ALGO=ipc2``; ``ipc`` = always; ``rccl`` =
        never.  Rank-independent (environment and backend only)."""
        mode = os.environ.get("MP4X_DM_LARGE", "auto").lower()
        if mode == "rccl" or not self.ipc_enabled or not flat.is_cuda:
            return False
        if flat.is_cuda and torch.cuda.is_current_stream_capturing():
            return False
        if mode != "ipc" and self.backend == "nccl" and self.algo not in ("ipc2", "ipc"):
            return False
        return self.ipc() is not None and self.ipc_large() is not None

    def _ipc_small_ok(self, flat: torch.Tensor, nbytes: int) -> bool:
        """The IPC copy-plan tier for broadcast / scatter / gather: up to the two-shot size, schedule
        not forced.  (Alignment and buffer fit are checked by IpcAllreduce, rank-independently.)"""
        if self.algo not in ("", "auto") or nbytes > self.ipc_twoshot_max or not self.ipc_enabled:
            return False
        if flat.is_cuda and torch.cuda.is_current_stream_capturing() and \
                (self._ipc_obj is None or self._ipc_obj._epoch_dev is None):
            return False
        return self.ipc() is not None

    def reduce(self, arr: torch.Tensor, frm: int, to: int, operator, operand, root: int, memo: bool = False):
        """``memo`` (the public API's full path): memoise the latency tier's launch (the staged IPC
        allreduce, which a reduce may run: non-root results are unspecified) for
        ProcessCommSlave.reduceArray's fast path."""
        flat = self._flat(arr)
        view = flat[frm:to]
        if view.numel() == 0:
            return arr
        op = self._op(operator, view)
        nbytes = view.numel() * view.element_size()
        t = self._root_tuned("reduce", view, op)
        if t == "rccl" and self.rccl_ok(op, view.dtype):
            self._count("reduce.rccl")
            self.coll.reduce(view, root, op.code)
            return arr
        if t == "ipc" and self._ipc_ok(op, view.dtype, nbytes) and self.ipc() is not None:
            from .ipc import TWOSHOT
            peers = self._ipc_obj.registered(view) if self._zc else None
            if peers is not None:
                self._count("reduce.ipc_zc")
                self._ipc_obj.allreduce_registered(view, op, peers)
                return arr
            inst = self.ipc_large() if nbytes > self.ipc_twoshot_max else self._ipc_obj
            if inst is not None:
                self._count("reduce.ipc2")
                inst.allreduce(view, op, algo=TWOSHOT)
                return arr
        if t == "a2a":
            self._count("reduce.a2a")
            froms, tos, _ = CommUtils.even_split(frm, to, self.p)
            self._reduce_scatter_a2a(flat, froms, tos, op)
            self.gather(flat, froms, tos, root)
            return arr
        if self.algo in ("", "auto") and nbytes > self.ipc_oneshot_max and self._zc_ok(flat) and \
                self._ipc_ok(op, view.dtype, nbytes) and not capturing_now():
            peers = self._ipc_obj.registered(view)
            if peers is not None:
                # a registered tensor (collective fact): the zero-copy two-shot, one kernel at any
                # size; non-root results are unspecified by the reduce contract
                self._count("reduce.ipc_zc")
                self._ipc_obj.allreduce_registered(view, op, peers)
                return arr
        if self.algo in ("", "auto") and self._ipc_ok(op, view.dtype, nbytes) and self._ipc_small_ok(flat, nbytes):
            # latency tier: the IPC allreduce kernels (non-root results are unspecified by the
            # reduce contract, ProcessCommSlave.java:1390-1421, so every rank may receive the sum)
            from .ipc import ONESHOT, TWOSHOT
            one = nbytes <= self._oneshot_limit()          # (the allreduce's crossover: two ranks, 4 MiB)
            self._count("reduce.ipc1" if one else "reduce.ipc2")
            self._ipc_obj.allreduce(view, op, algo=ONESHOT if one else TWOSHOT)
            if memo and self._fast_ar is not None and view.is_cuda and not capturing_now():
                self._fast_remember(arr, frm, to, operator, operand, 1.0, view, op, "ipc1" if one else "ipc2",
                                    kind="reduce")
            return arr
        if self.algo in ("", "auto") and self._ipc_ok(op, view.dtype, nbytes) and self._dm_large_ok(flat):
            from .ipc import TWOSHOT          # no RCCL underneath: the piecewise IPC two-shot
            self._count("reduce.ipc2")
            self.ipc_large().allreduce(view, op, algo=TWOSHOT)
            return arr
        sel = self.select("reduce", nbytes, op, view.dtype) if self.algo != "composite" else "a2a"
        if sel == "ipc2" and not capturing_now() and self.ipc() is not None:
            # an op RCCL cannot reduce, above the direct tier: the piecewise IPC two-shot
            inst = self.ipc_large() if nbytes > self.ipc_twoshot_max else self._ipc_obj
            if inst is not None:
                from .ipc import TWOSHOT
                self._count("reduce.ipc2")
                inst.allreduce(view, op, algo=TWOSHOT)
                return arr
        if sel == "rccl":
            self._count("reduce.rccl")
            self.coll.reduce(view, root, op.code)
        else:   # reduce-scatter + gather (reference reduceArray composition, ProcessCommSlave.java:1390-1421)
            self._count("reduce.a2a")
            froms, tos, _ = CommUtils.even_split(frm, to, self.p)
            self._reduce_scatter_a2a(flat, froms, tos, op)
            self.gather(flat, froms, tos, root)
        return arr

    # ================================================================== gather / scatter (p2p)
    def gather(self, arr: torch.Tensor, froms, tos, root: int, memo: bool = False):
        flat = self._flat(arr)
        r = self.rank
        t = self._root_tuned("gather", flat[froms[0]:tos[-1]], None)
        if self.algo in ("", "auto") and t != "p2p" and self._zc_ok(flat) and \
                (tos[-1] - froms[0]) * flat.element_size() > self.ipc_oneshot_max and \
                self._ipc_obj.gather_registered(flat, froms, tos, root):
            self._count("gather.ipc_zc")        # registered tensors: the root pulls from the peers' own
            return arr
        if t == "ipc" and self.ipc() is not None and self.ipc_large() is not None and \
                self.ipc_large().gather_large(flat, froms, tos, root):
            self._count("gather.ipc_large")
            return arr
        if t != "p2p" and self._ipc_small_ok(flat, (tos[-1] - froms[0]) * flat.element_size()) and \
                self._plan_memo(memo, "gather", arr, (tuple(froms), tuple(tos), root),
                                lambda: self._ipc_obj.gather(flat, froms, tos, root)):
            self._count("gather.ipc")
            return arr
        if t != "p2p" and self._dm_large_ok(flat) and self.ipc_large().gather_large(flat, froms, tos, root):
            self._count("gather.ipc_large")
            return arr
        self._count("gather")
        if r == root:
            self.coll.p2p([], [(flat[froms[j]:tos[j]], j) for j in range(self.p) if j != r and tos[j] > froms[j]])
        elif tos[r] > froms[r]:
            self.coll.p2p([(flat[froms[r]:tos[r]], root)], [])
        return arr

    def scatter(self, arr: torch.Tensor, froms, tos, root: int, memo: bool = False):
        flat = self._flat(arr)
        r = self.rank
        t = self._root_tuned("scatter", flat[froms[0]:tos[-1]], None)
        if self.algo in ("", "auto") and t != "p2p" and self._zc_ok(flat) and \
                (tos[-1] - froms[0]) * flat.element_size() > self.ipc_oneshot_max and \
                self._ipc_obj.scatter_registered(flat, froms, tos, root):
            self._count("scatter.ipc_zc")       # registered tensors: every rank pulls from the root's
            return arr
        if t == "ipc" and self.ipc() is not None and self.ipc_large() is not None and \
                self.ipc_large().scatter_large(flat, froms, tos, root):
            self._count("scatter.ipc_large")
            return arr
        if t != "p2p" and self._ipc_small_ok(flat, (tos[-1] - froms[0]) * flat.element_size()) and \
                self._plan_memo(memo, "scatter", arr, (tuple(froms), tuple(tos), root),
                                lambda: self._ipc_obj.scatter(flat, froms, tos, root)):
            self._count("scatter.ipc")
            return arr
        if t != "p2p" and self._dm_large_ok(flat) and self.ipc_large().scatter_large(flat, froms, tos, root):
            self._count("scatter.ipc_large")
            return arr
        self._count("scatter")
        if r == root:
            self.coll.p2p([(flat[froms[j]:tos[j]], j) for j in range(self.p) if j != r and tos[j] > froms[j]], [])
        elif tos[r] > froms[r]:
            self.coll.p2p([], [(flat[froms[r]:tos[r]], root)])
        return arr
