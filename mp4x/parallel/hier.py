"""Node-aware (hierarchical) allreduce for jobs that span several MI355X nodes.

The reference is a multi-HOST library: its slaves sit on different machines and every
collective crosses the network (/root/reference/README.md:300, ring RS + AG in
ProcessCommSlave.java:1329-1373).  mp4x runs one process per GPU; inside a node the GPUs share a
full xGMI mesh (7 point-to-point links per GPU), across nodes there is only the network.  A flat
RCCL ring over all ranks sends every byte over the slowest hop; this schedule instead keeps the
network traffic to 1/L of the message per rank (L = GPUs per node):

    1. intra-node reduce-scatter over xGMI   (IPC direct RS kernel, csrc/runtime/ipc.hip)
       -> local rank i holds its node's partial sum of chunk i;
    2. inter-node allreduce of chunk i among the ranks with local index i on every node
       (RCCL on a sub-communicator; L such communicators run at once, one NIC each);
    3. intra-node all-gather over xGMI      (IPC copy-plan kernel).

Messages are processed in pieces of ``MP4X_HIER_PIECE_BYTES`` (rank-independent, default
256 MiB) and pipelined: the inter-node allreduce of piece k runs on RCCL's stream while the
intra-node reduce-scatter of piece k+1 runs on the compute stream (xGMI and network busy at
once).  The fused 1/p average is applied to the chunk between steps 2 and 3 (1/L of the data).

Which ranks share a node is decided from ``MP4X_NODE_ID`` or the host name, exchanged over the
control plane; ``MP4X_SIM_NODE_SIZE=k`` simulates nodes of k consecutive ranks (tests and
one-GPU rehearsals).  A node whose IPC mesh cannot be built (or fails the exact-pattern check
run once at setup, agreed by every rank) runs steps 1 and 3 over its local process group
instead — the chunking is identical, so nodes may mix the two forms.
"""
from __future__ import annotations

import logging
import os
import socket
from typing import List, Optional

import torch
import torch.distributed as dist

from ..exceptions import Mp4jException
from ..operators import OpCode

LOG = logging.getLogger("mp4x.hier")


def node_id(rank: int) -> str:
    """The node a rank runs on: ``MP4X_SIM_NODE_SIZE`` simulation, ``MP4X_NODE_ID``, host name."""
    sim = os.environ.get("MP4X_SIM_NODE_SIZE")
    if sim:
        return f"sim-node-{rank // max(1, int(sim))}"
    return os.environ.get("MP4X_NODE_ID") or socket.gethostname()


class NodeLayout:
    """Ranks grouped by node (pure; unit-tested on CPU).  ``ids[r]`` = node id of rank r."""

    def __init__(self, ids: List[str]):
        order = list(dict.fromkeys(ids))                       # nodes in first-rank order
        self.ids = list(ids)
        self.nodes: List[List[int]] = [[r for r, x in enumerate(ids) if x == n] for n in order]
        self.node_of = [order.index(x) for x in ids]
        self.local_index = [self.nodes[self.node_of[r]].index(r) for r in range(len(ids))]

    @property
    def multi_node(self) -> bool:
        return len(self.nodes) > 1

    @property
    def local_size(self) -> int:
        return len(self.nodes[0]) if self.nodes else 0

    def hier_ok(self) -> bool:
        """Two or more nodes with the same number (>= 2) of ranks each."""
        return self.multi_node and self.local_size >= 2 and all(len(n) == self.local_size for n in self.nodes)

    def cross_groups(self) -> List[List[int]]:
        """Group i = the rank with local index i on every node, in node order."""
        return [[node[i] for node in self.nodes] for i in range(self.local_size)]


def chunk_bounds(lo: int, hi: int, es: int, L: int):
    """``L`` chunks of ``[lo, hi)`` (elements of ``es`` bytes) whose byte offsets from ``lo`` are
    16-byte multiples (the IPC kernels move 16-byte vectors); the last chunk takes the remainder.
    ``(hi - lo) * es`` must be a 16-byte multiple."""
    unit = max(1, 16 // es)
    units = (hi - lo) // unit
    per = units // L
    froms = [lo + i * per * unit for i in range(L)]
    tos = froms[1:] + [hi]
    return froms, tos


class _GroupServer:
    """Control-plane facade for a sub-mesh: the GLOBAL collectives of the master, filtered to
    ``members``.  Every rank of the job makes the same sequence of calls (the sub-meshes of all
    nodes are built and used in lockstep), so a global allgather serves every node at once."""

    def __init__(self, server, global_rank: int, members: List[int]):
        self._srv = server
        self._g = global_rank
        self._members = members

    def allgather_both(self, rank, obj):
        """(the members' values, every rank's values) of one global allgather: the IPC mesh setup
        agrees failures job-wide, so a node whose mesh fails raises at the same agreement point as
        every other node and the global calls that follow stay paired."""
        allv = self._srv.call("allgather_obj", self._g, obj)
        return [allv[m] for m in self._members], allv

    def call(self, method, rank, *args):
        if method == "allgather_obj":
            allv = self._srv.call("allgather_obj", self._g, *args)
            return [allv[m] for m in self._members]
        if method == "barrier":
            return self._srv.call("barrier", self._g)
        raise Mp4jException(f"sub-mesh control plane: {method} is not supported")


class _GroupComm:
    """What :class:`~mp4x.parallel.ipc.IpcAllreduce` needs from a communicator, for one node."""

    def __init__(self, comm, members: List[int], gpu_share: int):
        g = comm.rank
        self.rank = members.index(g)
        self.slaveNum = len(members)
        self.server = _GroupServer(comm.server, g, members)
        self.global_rank = g
        self.gpu_share = gpu_share

    def node_id(self) -> str:
        return node_id(self.global_rank)


class HierAllreduce:
    """Collective construction (every rank, same point).  ``engine``: the rank's DeviceEngine."""

    def __init__(self, engine, layout: NodeLayout):
        if not layout.hier_ok():
            raise Mp4jException(f"hierarchical allreduce needs >= 2 nodes of equal size >= 2: {layout.nodes}")
        self.engine = engine
        self.layout = layout
        r = engine.rank
        self.node = layout.nodes[layout.node_of[r]]
        self.L = len(self.node)
        self.li = layout.local_index[r]
        self.piece_bytes = int(os.environ.get("MP4X_HIER_PIECE_BYTES", 256 << 20)) // 16 * 16 or 16
        backend = engine.backend
        # every rank creates every group, in the same order (torch.distributed requirement)
        self._cross_pg = None
        for i, g in enumerate(layout.cross_groups()):
            pg = dist.new_group(ranks=g, backend=backend)
            if i == self.li:
                self._cross_pg = pg
        self._local_pg = None
        for node in layout.nodes:
            pg = dist.new_group(ranks=node, backend=backend)
            if r in node:
                self._local_pg = pg
        self.ipc = None
        self.stats = {"pieces": 0, "ipc_pieces": 0}
        self.selftest: Optional[dict] = None
        want_ipc = engine.device.type == "cuda" and os.environ.get("MP4X_IPC", "1") == "1" and 2 <= self.L <= 8
        share = 1
        if engine.device.type == "cuda":
            # processes per physical GPU across the whole job (one-GPU rehearsals): the sub-meshes
            # of different "nodes" then share one GPU's resident-block budget
            import ctypes
            from . import ipc as _ipc     # binds the runtime's signatures
            pci = ctypes.create_string_buffer(64)
            try:
                _ipc.native.hip().mp4x_device_pci_id(pci, 64)
            except Exception:   # noqa: BLE001 — an empty id only weakens the share estimate
                pass
            ids = engine.comm.server.call("allgather_obj", r, (socket.gethostname(), pci.value))
            share = max(ids.count(x) for x in ids)
        # the flag is rank-independent, so every rank takes part in the same setup collectives
        if want_ipc:
            from .ipc import IpcAllreduce
            try:
                self.ipc = IpcAllreduce(_GroupComm(engine.comm, self.node, share), nbytes=self.piece_bytes,
                                        tag="hier", slots=False)
                engine._adopt(self.ipc)
            except Exception as e:   # noqa: BLE001 — agreed inside the node's mesh setup
                LOG.warning("rank %d: intra-node IPC mesh unavailable (%s): local process group used", r, e)
                self.ipc = None
            self._self_test()

    # ------------------------------------------------------------------ setup check
    def _self_test(self) -> None:
        """One exact-pattern hierarchical allreduce (f32 SUM, 4 MiB) through the IPC sub-meshes;
        any wrong element or error on any rank drops IPC on every node (agreed through the
        control plane)."""
        from ..operators import Operators, for_dtype, DType
        eng = self.engine
        bad = None
        # every rank runs it (a node without a mesh takes the local-group form of steps 1 and 3)
        try:
            n = 1 << 20
            p, r = eng.p, eng.rank
            idx = torch.arange(n, device=eng.device, dtype=torch.int32).remainder_(61)
            t = (idx + r).to(torch.float32)
            self.allreduce(t, for_dtype(Operators.Float.SUM, DType.F32))
            torch.cuda.synchronize(eng.device)
            exp = (idx * p + p * (p - 1) // 2).to(torch.float32)
            nbad = int((t != exp).sum())
            bad = f"{nbad} wrong elements" if nbad else None
        except Exception as e:   # noqa: BLE001
            bad = f"{type(e).__name__}: {e}"
        allb = eng.comm.server.call("allgather_obj", eng.rank, bad)
        fails = [f"rank {i}: {b}" for i, b in enumerate(allb) if b]
        self.selftest = {"ok": not fails, "failures": fails, "ipc_nodes": None}
        if fails:
            LOG.warning("rank %d: hierarchical IPC self-test failed (%s): local process groups used", eng.rank, fails)
            # agreed job-wide: every rank is here.  Ordered teardown (every importer unmaps
            # before any owner frees, IpcAllreduce.close(collective=True)); a rank without a
            # sub-mesh joins the same global barrier
            if self.ipc is not None:
                try:
                    self.ipc.close(collective=True)
                except Exception as e:   # noqa: BLE001
                    LOG.warning("rank %d: closing the dropped sub-mesh: %s", eng.rank, e)
            else:
                eng.comm.server.call("barrier", eng.rank)
            self.ipc = None
        self.selftest["ipc_nodes"] = sum(1 for x in eng.comm.server.call("allgather_obj", eng.rank,
                                                                          self.ipc is not None) if x) // self.L

    # ------------------------------------------------------------------ the schedule
    def supports(self, view: torch.Tensor, op) -> bool:
        """Rank-independent: 16-byte message, an op both RCCL and the IPC kernels reduce."""
        if getattr(op, "is_custom", False) or (view.numel() * view.element_size()) % 16:
            return False
        from .ipc import SUPPORTED_DTYPES
        if view.dtype not in SUPPORTED_DTYPES or not self.engine.rccl_ok(op, view.dtype):
            return False
        return op.code == OpCode.SUM or (op.code in (OpCode.MAX, OpCode.MIN) and view.is_floating_point())

    def allreduce(self, view: torch.Tensor, op, scale: float = 1.0) -> None:
        """In place on a contiguous 1-D ``view``; ``scale`` (float dtypes) fused between the
        inter-node step and the all-gather."""
        es = view.element_size()
        n = view.numel()
        step = max(1, self.piece_bytes // es)
        pieces = [(a, min(n, a + step)) for a in range(0, n, step)]
        self.stats["pieces"] += len(pieces)
        pending = None                       # (work, chunk, froms, tos) of the previous piece
        for a, b in pieces:
            froms, tos = chunk_bounds(a, b, es, self.L)
            self._reduce_scatter(view, froms, tos, op)
            chunk = view[froms[self.li]:tos[self.li]]
            work = self._cross_start(chunk, op)
            if pending is not None:          # previous piece: its network step overlapped this RS
                self._finish(view, *pending, scale)
            pending = (work, chunk, froms, tos)
        if pending is not None:
            self._finish(view, *pending, scale)

    def _cross_start(self, chunk: torch.Tensor, op):
        if chunk.numel() == 0:
            return None
        from .coll import _RCCL_OPS
        return dist.all_reduce(chunk, op=_RCCL_OPS[op.code], group=self._cross_pg, async_op=True)

    def _finish(self, view, work, chunk, froms, tos, scale) -> None:
        if work is not None:
            work.wait()
        if scale != 1.0 and chunk.numel():
            if chunk.is_cuda:
                from ..ops.device_ops import scale_
                scale_(chunk, chunk, float(scale))
            else:
                chunk.mul_(scale)
        self._allgather(view, froms, tos)

    def _reduce_scatter(self, view, froms, tos, op) -> None:
        if self.ipc is not None and self.ipc.reduce_scatter(view, froms, tos, op):
            self.stats["ipc_pieces"] += 1
            return
        # local process group: the node's sum of the whole piece (own chunk used afterwards)
        from .coll import _RCCL_OPS
        dist.all_reduce(view[froms[0]:tos[-1]], op=_RCCL_OPS[op.code], group=self._local_pg)

    def _allgather(self, view, froms, tos) -> None:
        if self.ipc is not None and self.ipc.allgather(view, froms, tos):
            return
        for j, g in enumerate(self.node):
            if tos[j] > froms[j]:
                dist.broadcast(view[froms[j]:tos[j]], src=g, group=self._local_pg)

    def close(self) -> None:
        if self.ipc is not None:
            try:
                self.ipc.close()
            except Exception:   # noqa: BLE001
                pass
            self.ipc = None
