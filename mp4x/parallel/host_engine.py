"""Collective algorithms over the host data plane (numpy arrays, Python objects).

Algorithms follow the reference's schedules (Thakur/Rabenseifner/Gropp):

* ring allgather — p−1 steps, each block forwarded verbatim
  (ProcessCommSlave.java:694-737; here the received frame is re-sent without
  re-encoding);
* ring reduce-scatter — p−1 steps with reduce-on-receive, local value first
  (ProcessCommSlave.java:1329-1373, hot loop J/operand/DoubleOperand.java:196);
* binary-tree scatter on the :mod:`mp4x.utils.scatter_allocate` plan
  (ProcessCommSlave.java:1103-1159);
* gather on the same tree reversed — deterministic, no master pairing (the
  reference's ``dynamicBinaryTreeGather`` pairs ranks through the master's
  Exchanger, ProcessCommSlave.java:440-520);
* map variants of all of the above with per-key merge/reduce;
* recursive halving / doubling allreduce (Rabenseifner) for built-in operators: 2·log2(p)
  message rounds instead of the ring's 2(p−1), with the same bandwidth-optimal
  2(p−1)/p·S bytes per rank when p is a power of two; other p fold the excess ranks into
  their neighbours first.  ``ProcessCommSlave`` picks it by size and p
  (:func:`choose_allreduce`).

All routines work in place on the caller's array and are tag-matched, so no
master barrier is needed after every collective (the reference ends each ring
with ``barrier()``, :731, :1367).
"""
from __future__ import annotations

import os
from typing import Dict, List

import numpy as np

from ..operands import Operand
from ..utils.scatter_allocate import plan as scatter_plan
from . import wire


_NATIVE_REDUCE_MIN = 1 << 20
_NATIVE_DT = {np.dtype(np.float64): 0, np.dtype(np.float32): 1, np.dtype(np.int64): 2, np.dtype(np.int32): 3,
              np.dtype(np.int16): 4, np.dtype(np.int8): 5}   # enum mp4x_dtype
_native_lib = None


def _native_reduce(seg: np.ndarray, data, op) -> bool:
    """seg op= data through the host runtime's multi-threaded reduce (csrc/host/host_ops.cpp,
    the persistent fan-out pool): numpy's ufuncs run on one core, which made the reduce-on-
    receive the slowest stage of a large TCP allreduce.  Same element order and IEEE results as
    the numpy path; False when the operands do not qualify (custom operator, dtype, layout)."""
    global _native_lib
    if getattr(op, "is_custom", False) or getattr(op, "code", None) is None:
        return False
    dt = _NATIVE_DT.get(seg.dtype)
    if dt is None or int(op.dtype) != dt or not isinstance(data, np.ndarray) or data.dtype != seg.dtype:
        return False
    if not (seg.flags.c_contiguous and data.flags.c_contiguous) or data.size != seg.size:
        return False
    a, b = seg.ctypes.data, data.ctypes.data
    if a % seg.itemsize or b % seg.itemsize:          # frames land at any byte offset
        return False
    if _native_lib is None:
        try:
            from ..ops import native
            _native_lib = native.host()
        except Exception:      # noqa: BLE001 — not built: numpy path
            _native_lib = False
    if not _native_lib:
        return False
    from ..ops.native import ptr_array
    from ..utils.cpus import usable_cpus
    pp, keep = ptr_array([a, b])
    return _native_lib.mp4x_host_reduce(dt, int(op.code), a, pp, 2, seg.size, min(8, usable_cpus())) == 0


def _reduce_segment(arr, f: int, t: int, data, op) -> None:
    if isinstance(arr, np.ndarray):
        seg = arr[f:t]
        if seg.nbytes >= _NATIVE_REDUCE_MIN and _native_reduce(seg, data, op):
            return
        with np.errstate(over="ignore", invalid="ignore"):
            op.reduce_into(seg, data)
    else:
        for i in range(t - f):
            arr[f + i] = op.apply(arr[f + i], data[i])


def _write_segment(arr, f: int, t: int, data) -> None:
    if isinstance(arr, np.ndarray):
        arr[f:t] = data
    else:
        arr[f:t] = list(data)


RHD_MAX_BYTES_DEFAULT = 64 << 10


def choose_allreduce(p: int, nbytes: int, custom: bool) -> str:
    """``ring`` or ``rhd`` for a host allreduce of ``nbytes`` on ``p`` ranks.

    Custom (possibly non-commutative) operators keep the reference's ring.  Power-of-two p:
    RHD always (fewer rounds, same bytes).  Otherwise RHD only below ``MP4X_RHD_MAX_BYTES``
    (default 64 KiB; measured crossover for p = 6 lies between 8 and 256 KiB), where latency dominates the fold's extra full-message transfer.
    ``MP4X_HOST_ALGO=ring|rhd`` forces one.
    """
    import os
    forced = os.environ.get("MP4X_HOST_ALGO", "").lower()
    if forced in ("ring", "rhd"):
        return forced
    if custom or p <= 2:
        return "ring" if custom else "rhd"
    if p & (p - 1) == 0:
        return "rhd"
    lim = int(os.environ.get("MP4X_RHD_MAX_BYTES", RHD_MAX_BYTES_DEFAULT))
    return "rhd" if nbytes <= lim else "ring"


# MAP collectives: direct exchange over the mesh or the reference's ring.  Measured on the box
# (profiles/r2/host_map_algo_box.jsonl, 50k keys x float[16] per rank): direct 38 vs ring 78 ms at
# p = 4, but 112 vs 92 ms at p = 8 (p - 1 reader threads per process then contend for the GIL
# with the merging thread), so direct is the default up to MP4X_HOST_MAP_DIRECT_MAX_P = 4.
# MP4X_HOST_MAP_ALGO=ring | direct forces one.
_MAP_ALGO = os.environ.get("MP4X_HOST_MAP_ALGO", "auto")
_MAP_DIRECT_MAX_P = int(os.environ.get("MP4X_HOST_MAP_DIRECT_MAX_P", 4))


def _map_direct(p: int) -> bool:
    if p <= 2 or _MAP_ALGO == "ring":
        return False
    return _MAP_ALGO == "direct" or p <= _MAP_DIRECT_MAX_P


class HostEngine:
    def __init__(self, transport, rank: int, p: int):
        self.t = transport
        self.rank = rank
        self.p = p
        self._seq = 0

    def next_tag(self) -> int:
        self._seq += 1
        return self._seq

    # ================================================================== ARRAY
    def ring_allgather(self, arr, froms, tos, operand: Operand):
        p, r = self.p, self.rank
        if p == 1:
            return arr
        tag = self.next_tag()
        nxt, prv = (r + 1) % p, (r - 1) % p
        self.t.send(nxt, tag, wire.pack_segments(arr, [(r, froms[r], tos[r])], operand))
        for step in range(1, p):
            body = self.t.recv(prv, tag)
            for _, f, t, data in wire.unpack_segments(body, operand):
                _write_segment(arr, f, t, data)
            if step < p - 1:
                self.t.send(nxt, tag, [body])
        return arr

    def ring_reduce_scatter(self, arr, froms, tos, operand: Operand, op):
        p, r = self.p, self.rank
        if p == 1:
            return arr
        tag = self.next_tag()
        nxt, prv = (r + 1) % p, (r - 1) % p
        b0 = (r - 1) % p
        self.t.send(nxt, tag, wire.pack_segments(arr, [(r, froms[b0], tos[b0])], operand))
        for step in range(1, p):
            b = (r - step - 1) % p
            body = self.t.recv(prv, tag)
            for _, f, t, data in wire.unpack_segments(body, operand):
                _reduce_segment(arr, f, t, data, op)
            if step < p - 1:
                self.t.send(nxt, tag, wire.pack_segments(arr, [(r, froms[b], tos[b])], operand))
        return arr

    def rhd_allreduce(self, arr, frm: int, to: int, operand: Operand, op):
        """Recursive-halving reduce-scatter + recursive-doubling allgather on [frm, to).

        Ranks fold to the largest power of two p2 <= p: for r < 2(p − p2), odd r hands its
        range to r − 1 first and receives the result last.  Every block is reduced by exactly
        one rank and copied to the others, so all ranks end bit-identical.
        """
        p, r = self.p, self.rank
        if p == 1 or to <= frm:
            return arr
        t_fold, t_rs, t_ag = self.next_tag(), self.next_tag(), self.next_tag()
        p2 = 1 << (p.bit_length() - 1)
        rem = p - p2

        def real(v):
            return 2 * v if v < rem else v + rem

        def send(dst, tag, f, t):
            self.t.send(dst, tag, wire.pack_segments(arr, [(r, f, t)], operand))

        def recv(src, tag, reduce):
            for _, f, t, data in wire.unpack_segments(self.t.recv(src, tag), operand):
                if reduce:
                    _reduce_segment(arr, f, t, data, op)
                else:
                    _write_segment(arr, f, t, data)

        if r < 2 * rem:
            if r % 2:
                send(r - 1, t_fold, frm, to)
                recv(r - 1, t_fold, False)
                return arr
            recv(r + 1, t_fold, True)
            vr = r // 2
        else:
            vr = r - rem
        lo, hi = frm, to
        mask = p2 >> 1
        steps = []
        while mask:
            partner = real(vr ^ mask)
            mid = lo + (hi - lo) // 2
            keep, give = ((lo, mid), (mid, hi)) if not vr & mask else ((mid, hi), (lo, mid))
            if give[1] > give[0]:
                send(partner, t_rs, *give)
            if keep[1] > keep[0]:
                recv(partner, t_rs, True)
            steps.append((partner, give))
            lo, hi = keep
            mask >>= 1
        for partner, give in reversed(steps):
            if hi > lo:
                send(partner, t_ag, lo, hi)
            if give[1] > give[0]:
                recv(partner, t_ag, False)
            lo, hi = min(lo, give[0]), max(hi, give[1])
        if r < 2 * rem:
            send(r + 1, t_fold, frm, to)
        return arr

    def tree_scatter(self, arr, froms, tos, operand: Operand, root: int):
        """Root's segments [froms[i], tos[i]) land at rank i (in place)."""
        p, r = self.p, self.rank
        if p == 1:
            return arr
        tag = self.next_tag()
        tasks = scatter_plan(p, root)
        if r != root:
            src = next(t[0] for t in tasks if t[1] == r)
            body = self.t.recv(src, tag)
            for _, f, t, data in wire.unpack_segments(body, operand):
                _write_segment(arr, f, t, data)
        for (src, dst, rf, rt) in tasks:
            if src != r or dst == root:
                continue
            segs = [(i, froms[i], tos[i]) for i in range(rf, rt + 1)]
            self.t.send(dst, tag, wire.pack_segments(arr, segs, operand))
        return arr

    def tree_bcast(self, arr, frm: int, to: int, operand: Operand, root: int):
        """Whole-range broadcast down the scatter tree (latency path for small payloads)."""
        p, r = self.p, self.rank
        if p == 1:
            return arr
        tag = self.next_tag()
        tasks = scatter_plan(p, root)
        body = None
        if r != root:
            src = next(t[0] for t in tasks if t[1] == r)
            body = self.t.recv(src, tag)
            for _, f, t, data in wire.unpack_segments(body, operand):
                _write_segment(arr, f, t, data)
        for (src, dst, rf, rt) in tasks:
            if src != r or dst == root:
                continue
            parts = [body] if body is not None else wire.pack_segments(arr, [(root, frm, to)], operand)
            self.t.send(dst, tag, parts)
        return arr

    def tree_gather(self, arr, froms, tos, operand: Operand, root: int):
        """Rank i's [froms[i], tos[i]) lands at the root (in place), intermediates accumulate."""
        p, r = self.p, self.rank
        if p == 1:
            return arr
        tag = self.next_tag()
        tasks = scatter_plan(p, root)
        held = [(r, froms[r], tos[r])]
        for (src, dst, rf, rt) in reversed(tasks):
            if src != r or dst == root:
                continue
            body = self.t.recv(dst, tag)
            for rk, f, t, data in wire.unpack_segments(body, operand):
                _write_segment(arr, f, t, data)
                held.append((rk, f, t))
        if r != root:
            parent = next(t[0] for t in tasks if t[1] == r)
            self.t.send(parent, tag, wire.pack_segments(arr, held, operand))
        return arr

    # ================================================================== MAP
    def ring_allgather_maps(self, block: List[Dict], operand: Operand) -> List[List[Dict]]:
        """Every rank contributes a block (list of maps); returns blocks indexed by rank."""
        p, r = self.p, self.rank
        out: List[List[Dict]] = [None] * p
        out[r] = block
        if p == 1:
            return out
        tag = self.next_tag()
        if _map_direct(p):
            # direct: ONE encode, sent to every peer over its own mesh connection (the sender
            # never blocks: readers drain into mailboxes), decoded as it arrives — one step of
            # latency instead of p - 1 store-and-forward ring steps
            body = wire.pack_maps([(r, d) for d in block], operand)
            for j in range(1, p):
                self.t.send((r + j) % p, tag, body)
            for j in range(1, p):
                src = (r - j) % p
                got = wire.unpack_maps(self.t.recv(src, tag), operand)
                out[src] = [wire.to_dict(k, v) for _, k, v in got]
            return out
        nxt, prv = (r + 1) % p, (r - 1) % p
        self.t.send(nxt, tag, wire.pack_maps([(r, d) for d in block], operand))
        for step in range(1, p):
            body = self.t.recv(prv, tag)
            got = wire.unpack_maps(body, operand)
            origin = got[0][0] if got else (r - step) % p
            out[origin] = [wire.to_dict(k, v) for _, k, v in got]
            if step < p - 1:
                self.t.send(nxt, tag, [body])
        return out

    def ring_reduce_scatter_maps(self, blocks: List[List[Dict]], operand: Operand, op) -> List[Dict]:
        """blocks[b] = list of maps destined to rank b; returns this rank's reduced block.

        Reference: ``ringReduceScatter`` MAP branch / ``reduceScatterMapSpecial``
        (ProcessCommSlave.java:1212-1287, 1329-1373).  Inputs are copied, never
        cleared (the reference clears the caller's maps after sending,
        J/operand/DoubleOperand.java:130-134).
        """
        p, r = self.p, self.rank
        if _map_direct(p):
            # direct: block b goes straight to its owner b (p - 1 concurrent sends), the owner
            # merges the p - 1 received blocks in arrival-independent ring order — each merge
            # sees one rank's map, not the growing union a ring step re-encodes and forwards
            tag = self.next_tag()
            for j in range(1, p):
                b = (r + j) % p
                self.t.send(b, tag, wire.pack_maps([(r, d) for d in blocks[b]], operand))
            mine = [dict(d) for d in blocks[r]]
            for j in range(1, p):
                got = wire.unpack_maps(self.t.recv((r - j) % p, tag), operand)
                for jj, (_, keys, vals) in enumerate(got):
                    wire.merge_reduce(mine[jj], keys, vals, op)
            return mine
        local = [[dict(d) for d in blk] for blk in blocks]
        if p == 1:
            return local[0]
        tag = self.next_tag()
        nxt, prv = (r + 1) % p, (r - 1) % p
        b0 = (r - 1) % p
        self.t.send(nxt, tag, wire.pack_maps([(r, d) for d in local[b0]], operand))
        for step in range(1, p):
            b = (r - step - 1) % p
            body = self.t.recv(prv, tag)
            got = wire.unpack_maps(body, operand)
            for j, (_, keys, vals) in enumerate(got):
                wire.merge_reduce(local[b][j], keys, vals, op)
            if step < p - 1:
                self.t.send(nxt, tag, wire.pack_maps([(r, d) for d in local[b]], operand))
        return local[r]

    def tree_scatter_maps(self, blocks, operand: Operand, root: int) -> List[Dict]:
        """Root's ``blocks[i]`` (list of maps) goes to rank i."""
        p, r = self.p, self.rank
        if p == 1:
            return blocks[0]
        tag = self.next_tag()
        tasks = scatter_plan(p, root)
        have: Dict[int, List[Dict]] = {}
        if r == root:
            have = {i: blocks[i] for i in range(p)}
        else:
            src = next(t[0] for t in tasks if t[1] == r)
            body = self.t.recv(src, tag)
            for rk, keys, vals in wire.unpack_maps(body, operand):
                have.setdefault(rk, []).append(wire.to_dict(keys, vals))
        for (src, dst, rf, rt) in tasks:
            if src != r or dst == root:
                continue
            items = [(i, d) for i in range(rf, rt + 1) for d in have.get(i, [])]
            self.t.send(dst, tag, wire.pack_maps(items, operand))
        return have.get(r, [])

    def tree_gather_map(self, d: Dict, operand: Operand, root: int) -> Dict:
        """Union of every rank's map at root (duplicate key: one value survives)."""
        p, r = self.p, self.rank
        if p == 1:
            return d
        tag = self.next_tag()
        tasks = scatter_plan(p, root)
        acc = dict(d)
        for (src, dst, rf, rt) in reversed(tasks):
            if src != r or dst == root:
                continue
            body = self.t.recv(dst, tag)
            for _, keys, vals in wire.unpack_maps(body, operand):
                acc.update(wire.to_dict(keys, vals))
        if r != root:
            parent = next(t[0] for t in tasks if t[1] == r)
            self.t.send(parent, tag, wire.pack_maps([(r, acc)], operand))
        return acc

    def allgather_bytes(self, payload: bytes) -> List[bytes]:
        """Every rank's opaque byte string, rank order, peer to peer over the mesh: one send to
        every peer (the readers drain into mailboxes, so no ordering between ranks can block),
        then one receive from every peer.  Used for the map key-dictionary rounds, so new key
        strings never travel through the master (the reference's master carries only control:
        J/rpc/Server.java:131-137; its map contents move slave to slave, ProcessCommSlave.java:
        1329-1373)."""
        p, r = self.p, self.rank
        out: List[bytes] = [b""] * p
        out[r] = payload
        if p == 1:
            return out
        tag = self.next_tag()
        for j in range(1, p):
            self.t.send((r + j) % p, tag, [payload])
        for j in range(1, p):
            src = (r - j) % p
            out[src] = bytes(self.t.recv(src, tag))
        return out

    def tree_bcast_obj(self, payload: bytes, root: int) -> bytes:
        """Broadcast an opaque byte string down the scatter tree."""
        p, r = self.p, self.rank
        if p == 1:
            return payload
        tag = self.next_tag()
        tasks = scatter_plan(p, root)
        if r != root:
            src = next(t[0] for t in tasks if t[1] == r)
            payload = bytes(self.t.recv(src, tag))
        for (src, dst, rf, rt) in tasks:
            if src == r and dst != root:
                self.t.send(dst, tag, [payload])
        return payload

    def dissemination_barrier(self) -> None:
        """O(log p) peer barrier without the master."""
        p, r = self.p, self.rank
        if p == 1:
            return
        tag = self.next_tag()
        k = 1
        while k < p:
            self.t.send((r + k) % p, tag, [b""])
            self.t.recv((r - k) % p, tag)
            k <<= 1
