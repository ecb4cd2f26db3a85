"""Sparse ``Map<String, T>`` collectives on the GPU (BASELINE config 4).

Reference semantics: ``allreduceMap`` = hash partition → ring reduce-scatter of per-owner
maps → ring allgather → merge (ProcessCommSlave.java:2053-2088); set/list specials on top
(ProcessCommSlave.java:1583-1720, 2099-2230).

Device design (one process per GPU):

* keys become dense, rank-consistent ids (:class:`KeyDictionary`, numbered in sync rounds);
  only keys a rank has never seen are exchanged (host allgather), so a steady-state embedding
  / histogram sync moves no strings at all, and the id sort runs over ``bits`` bits only;
* values live in one ``[n, dim]`` device tensor (``Map<String, float[]>`` rows);
* owner of a key = ``(uint64)id % p``; kernel K4b partitions keys AND rows by owner in one
  fused LDS-multisplit pass (stable, deterministic; the rocPRIM radix-sort K4 path remains
  as the fallback) and they are exchanged with ONE ragged all-to-all over RCCL (every link
  busy at once, no ring);
* each owner reduces its rows with the deterministic reduce-by-key kernel K5 (stable sort
  by id, one wave per key, rows combined in source-rank order);
* owned results are all-gathered; ownership is disjoint, so the union needs no merge.

The tensor-level entry points (``allreduce_sparse``, ``set_union``, ``set_intersection``)
take int64 id tensors directly and are what a training loop should call.
"""
from __future__ import annotations

import itertools
import os
from collections.abc import MutableMapping
from typing import Dict, List, NamedTuple, Optional

import numpy as np
import torch

from ..operators import dtype_of_torch, for_dtype
from .wire import decode_keys, encode_keys  # noqa: F401 — the key codec of the map rounds


class KeyDictionary:
    """Rank-consistent DENSE ids for map keys (one dictionary per communicator).

    Ids are handed out in sync rounds (:func:`_sync_new_keys`, one control-plane allgather):
    every rank publishes the keys it has never seen, and every rank then numbers the union in
    the same order — rank 0's new keys in its first-seen order, then rank 1's not yet numbered,
    and so on — so all ranks agree with no coordinator and no hash collisions.  Dense ids keep
    the sort keys short: K5's radix sort only covers :attr:`bits` = the bit length of the
    largest id (3 onesweep passes instead of 8 for a million keys), and the owner ``id % p``
    deals keys round-robin over the ranks.  Keys may be any hashable (the reference's are
    ``String``)."""

    def __init__(self):
        self.id2key: List = []
        self.key2id: Dict = {}
        # (dict version, dict, base, ids, rows, {device copies}) of the last complete walk
        self._walk_cache = None
        # (key objects, ids) of the last complete walk: the native walk's position hint
        self._hint = None

    def unknown(self, keys) -> List:
        """Keys this rank has never numbered (first-seen order, de-duplicated)."""
        keys = keys if isinstance(keys, (list, tuple)) else list(keys)
        if all(map(self.key2id.__contains__, keys)):  # steady state: one C-level pass, no set built
            return []
        seen = set()
        out = []
        for k in keys:
            if k not in self.key2id and k not in seen:
                seen.add(k)
                out.append(k)
        return out

    def learn_round(self, proposals) -> None:
        """Number the union of one sync round's proposals (every rank passes the same list)."""
        from ..ops import native
        ext = native.hostmap_ext()
        if ext is not None:       # one dict probe per key (csrc/pyext/hostmap_ext.cpp learn_keys)
            got = ext.learn_keys(self.key2id, self.id2key, list(proposals))
            if isinstance(got, tuple):        # a large first round went into a presized dict
                self.key2id = got[1]
            return
        # C-level passes only (a first call numbers ~1M keys): order-preserving union of the
        # blocks, drop the known keys, number the rest in that order
        union = dict.fromkeys(itertools.chain.from_iterable(b for b in proposals if b))
        if self.key2id:
            new = [k for k in union if k not in self.key2id]
        else:
            new = list(union)
        base = len(self.id2key)
        self.key2id.update(zip(new, range(base, base + len(new))))
        self.id2key.extend(new)

    def ids(self, keys) -> List[int]:
        return [self.key2id[k] for k in keys]

    def lookup(self, keys) -> np.ndarray:
        """int64 ids of ``keys``, -1 where a key was never numbered (one C-level pass)."""
        keys = keys if isinstance(keys, (list, tuple)) else list(keys)
        return np.fromiter(map(self.key2id.get, keys, itertools.repeat(-1, len(keys))), dtype=np.int64,
                           count=len(keys))

    def id_array(self, keys) -> np.ndarray:
        """int64 ids of ``keys`` (one C-level pass)."""
        keys = keys if isinstance(keys, (list, tuple)) else list(keys)
        return np.fromiter(map(self.key2id.__getitem__, keys), dtype=np.int64, count=len(keys))

    def keys_of(self, ids: np.ndarray) -> List:
        """Keys of an int64 id array (vectorised through an object array cached per size)."""
        if getattr(self, "_obj_n", -1) != len(self.id2key):
            self._obj = np.asarray(self.id2key + [None], dtype=object)[:-1]   # (+None: 1-D even for tuples)
            self._obj_n = len(self.id2key)
        return self._obj[ids].tolist()

    @property
    def bits(self) -> int:
        return max(1, (len(self.id2key) - 1).bit_length())


def _dictionary(engine) -> KeyDictionary:
    d = getattr(engine, "_keydict", None)
    if d is None:
        d = engine._keydict = KeyDictionary()
    return d


def allgather_keys(engine, new: List) -> List[List]:
    """Every rank's key list, rank order — over the DATA plane: the host TCP mesh of the
    communicator (peer to peer, never through the master), the in-process hub for loopback
    ranks, the control plane only when neither exists."""
    if hasattr(engine.coll, "_exchange"):
        return engine.coll._exchange(list(new))
    if os.environ.get("MP4X_KEYS_VIA_MASTER") == "1":     # the round-2 path, kept for A/B records
        return engine.all_gather_object(list(new))
    host = getattr(engine.comm, "engine", None)
    if host is not None and hasattr(host, "allgather_bytes"):
        r = engine.rank
        mine = list(new)
        # this rank's own block is the list it already holds (no decode of its own bytes)
        return [mine if j == r else decode_keys(b) for j, b in enumerate(host.allgather_bytes(encode_keys(mine)))]
    return engine.all_gather_object(list(new))


def _sync_new_keys(engine, new: List) -> None:
    """One sync round: allgather (data plane, :func:`allgather_keys`) of every rank's unseen
    keys, numbered in rank order on every rank.  Collective — ranks with nothing new still take
    part.

    When the caller's device/host agreement round already numbered the new keys
    (``ProcessCommSlave._map_on_device`` sets ``engine._keys_presynced`` on EVERY rank), this
    round is skipped."""
    if getattr(engine, "_keys_presynced", False):
        engine._keys_presynced = False
        return
    _dictionary(engine).learn_round(allgather_keys(engine, new))


# ------------------------------------------------------------------ local kernels (GPU) / CPU twins
# Reduce-by-key of the device map collectives (K5): "sort" (default: deterministic, keys ascending
# per owner — K5d's direct addressing when the carried key range is dense enough (_dense_plan),
# else rocPRIM radix sort + run starts + the segmented reduce; both give the same result and
# order) or "hash" (K5h,
# csrc/kernels/sparse_hash.hip: open addressing, a row list per key, rows combined in input order —
# the same values bit for bit, 1.4-1.6x faster on config 4's owner rows; keys in table order,
# which depends on the CAS races of colliding keys).  A/B: profiles/r6/sparse/v3_*.
RBK_MODE = os.environ.get("MP4X_SPARSE_RBK", "sort").lower()
def _reduce_by_key(keys: torch.Tensor, vals: Optional[torch.Tensor], op, key_bits: Optional[int] = None,
                   dense=None):
    """``key_bits``: every key is in [0, 2**key_bits) (dense dictionary ids) — the radix sort
    covers those bits only.  ``dense`` = (base, stride, T) from :func:`_dense_plan`: K5d runs
    instead (no sort; the same result, order included) unless the keys turn out not dense."""
    if keys.is_cuda:
        from ..ops.device_ops import reduce_by_key
        if dense is not None and RBK_MODE != "hash" and (vals is None or not getattr(op, "is_custom", False)):
            from ..ops.device_ops import dense_reduce_by_key, hash_rbk_supported
            if vals is None or hash_rbk_supported(vals.dtype, int(op.code)):
                got = dense_reduce_by_key(keys, vals, int(op.code) if vals is not None else 0, *dense)
                if got is not None:
                    return got
        if vals is not None and RBK_MODE == "hash" and not getattr(op, "is_custom", False):
            from ..ops.device_ops import hash_rbk_supported, hash_reduce_by_key
            if hash_rbk_supported(vals.dtype, int(op.code)):
                return hash_reduce_by_key(keys, vals, int(op.code))
        return reduce_by_key(keys, vals, int(op.code) if vals is not None else 0, key_bits=key_bits)
    # CPU twin for the gloo test configuration only
    uk, inv, cnt = torch.unique(keys, sorted=True, return_inverse=True, return_counts=True)
    if vals is None:
        return uk, None, cnt.to(torch.int32)
    order = torch.argsort(inv, stable=True)
    out = torch.empty((uk.numel(),) + tuple(vals.shape[1:]), dtype=vals.dtype)
    vnp = vals.numpy()
    inv_np = inv.numpy()
    onp = out.numpy()
    seen = np.zeros(uk.numel(), dtype=bool)
    for j in order.numpy():
        u = inv_np[j]
        if not seen[u]:
            onp[u] = vnp[j]
            seen[u] = True
        else:
            row = np.array(onp[u], copy=True)
            op.reduce_into(row.reshape(-1), vnp[j].reshape(-1))
            onp[u] = row
    return uk, out, cnt.to(torch.int32)


def _owner(keys: torch.Tensor, p: int) -> torch.Tensor:
    """CPU twin of the device owner ``(uint64)id % p`` (ids are int64 two's complement)."""
    dest = torch.remainder(keys, p)
    wrap = (1 << 64) % p
    if wrap:
        dest = torch.where(keys < 0, torch.remainder(dest + wrap, p), dest)
    return dest


def _owner_order(keys: torch.Tensor, p: int):
    """(perm sorting rows by owner, per-owner counts) — kernels K4 + stable radix sort."""
    if keys.is_cuda:
        from ..ops.device_ops import key_owner, sort_pairs
        dest, hist = key_owner(keys, p)
        bits = max(1, int(p - 1).bit_length())
        _, perm = sort_pairs(dest, end_bit=bits)
        return perm, hist.to(torch.int64)
    dest = _owner(keys, p)
    perm = torch.argsort(dest, stable=True)
    return perm, torch.bincount(dest, minlength=p)


def _pack_by_owner(keys: torch.Tensor, vals: Optional[torch.Tensor], p: int, want_range: bool = False):
    """(keys, rows) in stable owner-major order + per-owner counts (``want_range``: followed by
    the smallest and largest key, as :func:`_owner_info` lays them out).

    GPU: one fused K4b launch chain (LDS multisplit, :func:`mp4x.ops.device_ops.partition_pack`);
    the sort-based K4 path remains for p beyond the fused kernel's LDS budget and on CPU.
    """
    if keys.is_cuda:
        from ..ops.device_ops import PACK_MAX_P, partition_pack
        if p <= PACK_MAX_P:
            sk, sv, counts, _ = partition_pack(keys, vals, p, want_range=want_range)
            return sk, sv, counts
    perm, hist = _owner_order(keys, p)
    skeys = _gather_rows(keys.view(-1, 1), perm).view(-1)
    svals = _gather_rows(vals, perm) if vals is not None else None
    return skeys, svals, (_owner_info(keys, hist) if want_range else hist)


def _gather_rows(x: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    if x.is_cuda:
        from ..ops.device_ops import gather_rows
        return gather_rows(x.contiguous(), idx)
    return x[idx]


# ------------------------------------------------------------------ IPC data plane for the sparse path
# The ragged exchanges of the map collectives as ONE copy-plan kernel each over the IPC mesh
# (csrc/runtime/ipc.hip k_ipc_copy_plan).  Every rank stages its rows and keys in its own IPC
# buffer as two regions — the rows (16-byte multiples), then the keys as 16-byte {key, 0} vectors
# from a rank-independent offset — so every block is whole 16-byte vectors whatever the row
# counts; the receiver pulls rows straight into a contiguous row block and keys into a key block
# (one small pass turns those into int64 keys).  All-to-all-v: each rank pulls its block from
# every peer at once (every xGMI link busy; no RCCL all_to_all).  All-gather-v: every rank pulls
# every peer's owned result.  The staging copy runs right before the plan, on the stream joined to
# the communicator's order: the previous collective of the instance has finished on this rank, and
# its end barrier means every peer has finished reading this buffer too.  The grid is sized from
# the full count matrix, which every rank knows, so every rank launches the same grid.
_SPARSE_IPC = os.environ.get("MP4X_SPARSE_IPC", "1") == "1"


def _row_bytes(vals: Optional[torch.Tensor]) -> int:
    """Row bytes (0 without rows), or -1 when rows are not a whole number of 16-byte vectors."""
    rb = 0 if vals is None else int(np.prod(vals.shape[1:], dtype=np.int64)) * vals.element_size()
    return rb if rb % 16 == 0 else -1


def _ipc_inst(engine, need_bytes: int):
    """The IPC instance whose staging buffer fits ``need_bytes`` (rank-independent), or None."""
    if need_bytes <= engine._ipc_obj.nbytes:
        return engine._ipc_obj
    big = engine.ipc_large()
    return big if big is not None and need_bytes <= big.nbytes else None


def _sparse_ipc_ok(engine, keys: torch.Tensor) -> bool:
    """Rank-independent: environment, device kind, capture state and the mesh."""
    from ..ops.native import capturing_now
    return _SPARSE_IPC and keys.is_cuda and getattr(engine, "ipc_enabled", False) and \
        engine.coll.__class__.__name__ == "TorchColl" and not capturing_now() and engine.ipc() is not None


def _split_exchange(engine, keys, vals, rb: int, nmax: int, blocks, grid_rows: int, stage=None):
    """Stage (keys, rows) in this rank's buffer (rows at vector 0, keys at ``nmax * V``) and run
    one copy plan; ``blocks`` = [(peer, src_row, rows)] pulled in order; ``grid_rows`` = the
    largest block of ANY rank (the plan's grid must be rank-independent).  ``stage(rows_ptr,
    keys16_ptr)`` writes the staged layout itself (the owner exchange's pack scatters straight
    into the buffer); default: a copy of ``keys`` / ``vals``.  Returns the received (keys, rows),
    or None when the largest rank's payload does not fit (rank-independent)."""
    from ..ops.device_ops import keys_from16, stage_split
    inst = _ipc_inst(engine, nmax * (rb + 16))
    if inst is None:
        return None
    V = rb // 16
    koff = nmax * V                               # first key vector: the same on every rank
    inst._launch_stream()                         # the communicator's stream order, then stage
    base = inst._data.value
    if stage is not None:
        stage(base, base + koff * 16)
    else:
        stage_split(keys.contiguous(), vals.contiguous() if vals is not None else None, base, base + koff * 16)
    total = sum(c for _, _, c in blocks)
    out = torch.empty(total * (rb + 16), dtype=torch.uint8, device=keys.device)
    pulls, off = [], 0
    for j, s0, c in blocks:
        if c:
            if V:
                pulls.append((s0 * V, off * V, c * V, j))
            pulls.append((koff + s0, total * V + off, c, j))
        off += c
    grid = grid_rows * max(V, 1)
    if grid:
        inst._plan([], pulls, None, out.data_ptr() if pulls else None, grid)
    rk = keys_from16(out[total * rb:])
    rv = None
    if vals is not None:
        rv = out[:total * rb].view(vals.dtype).view((total,) + tuple(vals.shape[1:]))
    return rk, rv


def _ipc_alltoallv(engine, skeys, svals, mat: List[List[int]], stage=None):
    """Owner exchange over the IPC mesh; ``mat[i][j]`` = rows rank i sends to rank j.  Returns
    (keys, rows) received in source-rank order, or None when rows are not 16-byte vectors or the
    largest rank's payload exceeds the staging buffers (both rank-independent).  ``stage``: see
    :func:`_split_exchange` (then ``skeys`` / ``svals`` only give the device, shapes and dtype)."""
    rb = _row_bytes(svals)
    if rb < 0:
        return None
    p, r = engine.p, engine.rank
    blocks = [(j, sum(mat[j][:r]), mat[j][r]) for j in range(p)]     # rank j's block for this rank
    got = _split_exchange(engine, skeys, svals, rb, max(sum(row) for row in mat), blocks,
                          max(max(row) for row in mat), stage)
    if got is not None:
        engine._count("sparse.a2a.ipc")
    return got


def _ipc_rows_alltoallv(engine, rows: torch.Tensor, mat: List[List[int]]):
    """Dense all-to-all-v of ``rows`` (uint8 [n, rb], rb a 16-byte multiple, grouped by
    destination) over the IPC mesh — ``alltoallArray``'s expert-parallel style routing as ONE
    copy-plan kernel: this rank stages its whole send buffer, every rank pulls its block from
    every peer at once.  ``mat[i][j]`` = rows rank i sends to rank j (every rank knows it).
    Returns the received rows in source-rank order, or None when the largest rank's payload
    does not fit the staging buffers (rank-independent)."""
    p, r = engine.p, engine.rank
    rb = rows.shape[1]
    v = rb // 16
    inst = _ipc_inst(engine, max(sum(row) for row in mat) * rb)
    if inst is None:
        return None
    n = sum(mat[r])
    src = rows if rows.data_ptr() % 16 == 0 else rows.clone()
    stage = [(0, 0, n * v, 0)] if n else []
    pulls, off = [], 0
    for j in range(p):
        s0 = sum(mat[j][:r])                      # rank j's block for this rank, in its buffer
        if mat[j][r]:
            pulls.append((s0 * v, off * v, mat[j][r] * v, j))
        off += mat[j][r]
    out = torch.empty((off, rb), dtype=torch.uint8, device=rows.device)
    glen = max(sum(row) for row in mat) * v       # sizes the grid: rank-independent
    if glen:
        inst._plan(stage, pulls, src.data_ptr() if stage else None, out.data_ptr() if pulls else None, glen)
    engine._count("all_to_all_v.ipc")
    return out


def _ipc_allgatherv(engine, keys, vals, sizes: List[int]):
    """Every rank's (keys, rows), rank order, over the IPC mesh (see above), or None."""
    rb = _row_bytes(vals)
    if rb < 0:
        return None
    got = _split_exchange(engine, keys, vals, rb, max(sizes), [(j, 0, sz) for j, sz in enumerate(sizes)], max(sizes))
    if got is not None:
        engine._count("sparse.allgatherv.ipc")
    return got


def _host_counts(engine) -> bool:
    """Small count vectors of GPU-resident data go over the host mesh when no RCCL is underneath
    (gloo standing in on device tensors stages even 8 integers through a device sync + host copy
    + TCP round per call)."""
    return engine.backend == "gloo" and engine.device.type == "cuda" and \
        getattr(engine.comm, "engine", None) is not None and hasattr(engine.comm.engine, "allgather_bytes")


def _count_matrix(engine, hist: torch.Tensor) -> List[List[int]]:
    """Every rank's per-destination row counts (one all-gather, one host sync)."""
    if _host_counts(engine):
        blobs = engine.comm.engine.allgather_bytes(hist.to(torch.int64).cpu().numpy().tobytes())
        return [np.frombuffer(b, dtype=np.int64).tolist() for b in blobs]
    ts = [torch.empty_like(hist) for _ in range(engine.p)]
    engine.coll.all_gather(ts, hist)
    return torch.stack(ts).tolist()


def _owner_info(keys: torch.Tensor, hist: torch.Tensor) -> torch.Tensor:
    """This rank's count-matrix row plus its key range: hist[p] | min | max (0 | 0 when empty).
    The range rides the count exchange, so every rank learns the received keys' bit width for
    free and the reduce-by-key's radix sort runs over those bits only.  (The fused GPU pack
    produces this row itself: ``_pack_by_owner(..., want_range=True)``.)"""
    hist = hist.to(torch.int64)
    if keys.numel() == 0:
        return torch.cat([hist, hist.new_zeros(2)])
    mn, mx = torch.aminmax(keys)
    return torch.cat([hist, mn.view(1), mx.view(1)])


class KeyRange(NamedTuple):
    """Every rank's keys lie in [lo, hi] (carried by the count exchange); ``bits`` bounds them for
    the radix sort (None when a key is negative)."""
    lo: int
    hi: int
    bits: Optional[int]


def _split_info(rows: List[List[int]], p: int, with_range: bool = False):
    """(count matrix, key bits of every rank's keys or None[, KeyRange]) from the
    :func:`_owner_info` rows."""
    mat = [r[:p] for r in rows]
    lo = min(r[p] for r in rows)
    hi = max(r[p + 1] for r in rows)
    bits = max(1, int(hi).bit_length()) if lo >= 0 else None
    bits = bits if bits is not None and bits <= 63 else None
    return (mat, bits, KeyRange(lo, hi, bits)) if with_range else (mat, bits)


# K5d pays ~12 bytes of table per slot (init, count, compact passes); measured on config 4's owner
# rows it beats the sort up to ~26 slots per row (0.096 vs 0.140 ms; profiles/r6/sparse/k5d_*)
DENSE_FACTOR = float(os.environ.get("MP4X_SPARSE_DENSE_FACTOR", 32.0))
DENSE_MAX_SLOTS = 1 << 26


def _bits_range(key_bits: Optional[int]) -> Optional["KeyRange"]:
    """The key range a caller's ``key_bits`` promises ([0, 2**key_bits)), or None."""
    return KeyRange(0, (1 << int(key_bits)) - 1, int(key_bits)) if key_bits else None


def _dense_plan(rng: Optional["KeyRange"], p: int, rkeys: torch.Tensor):
    """K5d's (base, stride, T) for an owner's received keys — every key k has k % p == this
    owner, so k // p - lo // p indexes a table of T slots — when that table is at most
    ``DENSE_FACTOR`` x the rows (dense or moderately sparse ids: dictionary numbering, feature
    ids, config 4's ranges) and ``DENSE_MAX_SLOTS``, else None."""
    n = rkeys.shape[0]
    if rng is None or rng.lo < 0 or n == 0 or not rkeys.is_cuda or DENSE_FACTOR <= 0:
        return None
    base = rng.lo // p
    T = rng.hi // p - base + 1
    return (base, p, T) if T <= min(DENSE_FACTOR * n, DENSE_MAX_SLOTS) else None


# ------------------------------------------------------------------ tensor-level API
def _exchange_by_owner(engine, keys: torch.Tensor, vals: Optional[torch.Tensor]):
    """(received keys, received rows, key range): the ranks' :class:`KeyRange` when the count
    exchange carried it (the IPC path), else None."""
    p = engine.p
    ipc = _sparse_ipc_ok(engine, keys)
    rng = None
    from ..ops.device_ops import PACK_MAX_P
    if ipc and p <= PACK_MAX_P and _row_bytes(vals) >= 0:
        # K4b in two halves: count, exchange the counts (they pick the staging instance), then
        # scatter the owner-sorted rows and keys straight into the staging buffer
        from ..ops.device_ops import partition_count, partition_scatter
        keys = keys.contiguous()
        vals = vals.contiguous() if vals is not None else None
        pc = partition_count(keys, p)
        mat, _, rng = _split_info(_count_matrix(engine, pc.info), p, with_range=True)
        got = _ipc_alltoallv(engine, keys, vals, mat,
                             stage=lambda rows_ptr, keys16_ptr: partition_scatter(pc, vals, rows_ptr, keys16_ptr, 2))
        if got is not None:
            return got[0], got[1], rng
        skeys = torch.empty_like(keys)                 # too large for the staging buffers
        svals = torch.empty_like(vals) if vals is not None else None
        partition_scatter(pc, vals, svals.data_ptr() if vals is not None else 0, skeys.data_ptr())
        send = mat[engine.rank]
        recv = [mat[j][engine.rank] for j in range(p)]
    elif ipc:
        skeys, svals, hist = _pack_by_owner(keys, vals, p, want_range=True)
        mat, _, rng = _split_info(_count_matrix(engine, hist), p, with_range=True)
        got = _ipc_alltoallv(engine, skeys, svals, mat)
        if got is not None:
            return got[0], got[1], rng
        send = mat[engine.rank]
        recv = [mat[j][engine.rank] for j in range(p)]
    else:
        skeys, svals, hist = _pack_by_owner(keys, vals, p)
        recv_counts = torch.empty_like(hist)
        engine.coll.all_to_all_single(recv_counts, hist)
        send, recv = torch.stack([hist, recv_counts]).tolist()      # one host sync for both
    rkeys = torch.empty(sum(recv), dtype=keys.dtype, device=keys.device)
    engine.coll.all_to_all_single(rkeys, skeys, recv, send)
    rvals = None
    if vals is not None:
        rvals = torch.empty((sum(recv),) + tuple(vals.shape[1:]), dtype=vals.dtype, device=vals.device)
        engine.coll.all_to_all_single(rvals, svals, recv, send)
    return rkeys, rvals, rng


def _row_counts(engine, n: int, device) -> List[int]:
    if device.type == "cuda" and _host_counts(engine):
        return [int(np.frombuffer(b, dtype=np.int64)[0])
                for b in engine.comm.engine.allgather_bytes(np.array([n], dtype=np.int64).tobytes())]
    t = torch.tensor([n], dtype=torch.int64, device=device)
    ts = [torch.empty_like(t) for _ in range(engine.p)]
    engine.coll.all_gather(ts, t)
    return torch.cat(ts).tolist()                  # one host sync, not p


def _allgather_v(engine, t: torch.Tensor, sizes: Optional[List[int]] = None) -> torch.Tensor:
    """Rows of every rank, rank order.  ONE all_gather_into_tensor of the rows padded to the
    largest count, then (unequal counts only) one multi-segment copy (K3) compacting the p
    blocks on the GPU — no list of p outputs and no torch.cat (2.3 TB/s on the box)."""
    p = engine.p
    if sizes is None:
        sizes = _row_counts(engine, t.shape[0], t.device)
    m = max(sizes) if sizes else 0
    tail = tuple(t.shape[1:])
    total = sum(sizes)
    if m == 0:
        return torch.empty((0,) + tail, dtype=t.dtype, device=t.device)
    t = t.contiguous()
    if all(s == m for s in sizes):
        out = torch.empty((total,) + tail, dtype=t.dtype, device=t.device)
        engine.coll.all_gather_into_tensor(out, t)
        return out
    pad = t
    if t.shape[0] != m:
        pad = torch.empty((m,) + tail, dtype=t.dtype, device=t.device)
        if t.shape[0]:
            pad[:t.shape[0]] = t
    gath = torch.empty((p * m,) + tail, dtype=t.dtype, device=t.device)
    engine.coll.all_gather_into_tensor(gath, pad)
    w = pad[0].numel()
    if t.is_cuda:
        from ..ops.device_ops import segment_copy_
        out = torch.empty((total,) + tail, dtype=t.dtype, device=t.device)
        segs, off = [], 0
        for i, s in enumerate(sizes):
            segs.append((off * w, i * m * w, s * w))
            off += s
        segment_copy_(out.view(-1), gath.view(-1), segs)
        return out
    return torch.cat([gath[i * m:i * m + s] for i, s in enumerate(sizes)], 0)


def allreduce_sparse(engine, keys: torch.Tensor, vals: torch.Tensor, operator, key_bits: Optional[int] = None):
    """All ranks end with the op-reduction of every rank's (key, row) pairs, keys ascending per owner.

    ``keys`` int64 [n] (unique per rank), ``vals`` [n, dim] (or [n]).
    """
    squeeze = vals.dim() == 1
    v2 = vals.view(-1, 1) if squeeze else vals
    op = operator if getattr(operator, "is_custom", False) else for_dtype(operator, dtype_of_torch(vals.dtype))
    rkeys, rvals, rng = _exchange_by_owner(engine, keys, v2)
    uk, uv, _ = _reduce_by_key(rkeys, rvals, op, key_bits or (rng.bits if rng else None),
                               _dense_plan(rng or _bits_range(key_bits), engine.p, rkeys))
    sizes = _row_counts(engine, uk.shape[0], uk.device)     # one count round for keys AND rows
    got = _ipc_allgatherv(engine, uk, uv, sizes) if _sparse_ipc_ok(engine, uk) else None
    if got is not None:
        all_k, all_v = got
    else:
        all_k = _allgather_v(engine, uk, sizes)
        all_v = _allgather_v(engine, uv, sizes)
    return all_k, (all_v.view(-1) if squeeze else all_v)


OP_FIRST = 11     # native MP4X_FIRST: keep the first row of every key (K8 map merge)


def _dedupe_first(keys: torch.Tensor, vals: Optional[torch.Tensor], key_bits: Optional[int] = None):
    """K8: unique keys ascending, each with its FIRST row in input (= rank) order."""
    if keys.is_cuda:
        from ..ops.device_ops import reduce_by_key
        uk, uv, _ = reduce_by_key(keys, vals, OP_FIRST, key_bits=key_bits)
        return uk, uv
    uk, inv = torch.unique(keys, sorted=True, return_inverse=True)
    first = torch.full((uk.numel(),), keys.numel(), dtype=torch.int64)
    first.scatter_reduce_(0, inv, torch.arange(keys.numel()), "amin")
    return uk, (vals[first] if vals is not None else None)


def allgather_sparse(engine, keys: torch.Tensor, vals: torch.Tensor):
    """Every rank's (keys, rows) concatenated in rank order + the per-rank row counts."""
    sizes = _row_counts(engine, keys.shape[0], keys.device)
    got = _ipc_allgatherv(engine, keys, vals, sizes) if _sparse_ipc_ok(engine, keys) else None
    if got is not None:
        return got[0], got[1], sizes
    return _allgather_v(engine, keys, sizes), _allgather_v(engine, vals, sizes), sizes


def gather_sparse(engine, keys: torch.Tensor, vals: torch.Tensor, root: int, key_bits: Optional[int] = None):
    """Root receives every rank's pairs (grouped p2p, all links at once) and merges them with
    K8 (duplicate key: the lowest rank's row survives).  Non-root ranks get their input back."""
    sizes = _row_counts(engine, keys.shape[0], keys.device)
    r = engine.rank
    if r != root:
        sends = [(keys, root)] + ([(vals, root)] if vals.numel() else []) if sizes[r] else []
        engine.coll.p2p(sends, [])
        return keys, vals
    tail = tuple(vals.shape[1:])
    ks, vs, recvs = [], [], []
    for j in range(engine.p):
        if j == root:
            ks.append(keys)
            vs.append(vals)
            continue
        kb = torch.empty(sizes[j], dtype=keys.dtype, device=keys.device)
        vb = torch.empty((sizes[j],) + tail, dtype=vals.dtype, device=vals.device)
        ks.append(kb)
        vs.append(vb)
        if sizes[j]:
            recvs.append((kb, j))
            if vb.numel():
                recvs.append((vb, j))
    engine.coll.p2p([], recvs)
    return _dedupe_first(torch.cat(ks), torch.cat(vs), key_bits)


def broadcast_sparse(engine, keys: Optional[torch.Tensor], vals: Optional[torch.Tensor], root: int):
    """Root's (keys, rows) on every rank (shape/dtype travel over the control plane)."""
    meta = engine.all_gather_object(
        (int(keys.shape[0]), tuple(vals.shape[1:]), str(vals.dtype).replace("torch.", ""))
        if engine.rank == root else None)[root]
    n, tail, dt = meta
    dev = engine.device
    if engine.rank != root:
        keys = torch.empty(n, dtype=torch.int64, device=dev)
        vals = torch.empty((n,) + tuple(tail), dtype=getattr(torch, dt), device=dev)
    if n:
        engine.coll.broadcast(keys, root)
        if vals.numel():
            engine.coll.broadcast(vals, root)
    return keys, vals


def reduce_sparse(engine, keys: torch.Tensor, vals: torch.Tensor, operator, root: int,
                  key_bits: Optional[int] = None):
    """Owner exchange + K5 reduce-by-key, then the owner-disjoint pieces go to ``root``."""
    squeeze = vals.dim() == 1
    v2 = vals.view(-1, 1) if squeeze else vals
    op = operator if getattr(operator, "is_custom", False) else for_dtype(operator, dtype_of_torch(vals.dtype))
    rkeys, rvals, rng = _exchange_by_owner(engine, keys, v2)
    uk, uv, _ = _reduce_by_key(rkeys, rvals, op, key_bits or (rng.bits if rng else None),
                               _dense_plan(rng or _bits_range(key_bits), engine.p, rkeys))
    gk, gv = gather_sparse(engine, uk, uv, root, key_bits)    # disjoint owners: K8 dedupe is a no-op
    return gk, (gv.view(-1) if squeeze else gv)


def _set_counts(engine, ids: torch.Tensor):
    ids = torch.unique(ids) if not ids.is_cuda else _reduce_by_key(ids, None, None)[0]
    rkeys, _, rng = _exchange_by_owner(engine, ids, None)
    return _reduce_by_key(rkeys, None, None, rng.bits if rng else None, _dense_plan(rng, engine.p, rkeys))


def set_union(engine, ids: torch.Tensor) -> torch.Tensor:
    """K7 union of int64 id sets across ranks."""
    uk, _, _ = _set_counts(engine, ids)
    return _allgather_v(engine, uk)


def set_intersection(engine, ids: torch.Tensor) -> torch.Tensor:
    """K7 intersection: ids present on all p ranks (count == p after de-duplication)."""
    uk, _, cnt = _set_counts(engine, ids)
    return _allgather_v(engine, uk[cnt == engine.p])


def list_concat(engine, ids: torch.Tensor) -> torch.Tensor:
    """K7 concat = allgather-v in rank order."""
    return _allgather_v(engine, ids)


# ------------------------------------------------------------------ Map API
class TensorMap(MutableMapping):
    """The ``Dict[key, Tensor]`` a device map collective returns: a mapping VIEW over the
    result's (dense key ids, value rows) instead of one Python tensor object per key.

    Building a real dict costs one tensor view per key (~3 us each: 900k result keys of the
    BASELINE config-4 allreduce took seconds in the conversion alone); here a key's row view is
    made when it is accessed.  Behaves like a dict (lookup, ``in``, iteration in result order,
    ``len``, ``items``, ``==``, assignment / deletion through an overlay).  Passed back into a
    map collective unmodified, its ids and rows are used directly (no per-key work at all)."""

    def __init__(self, d: "KeyDictionary", ids, rows: torch.Tensor, shape):
        self._d = d
        # ids stay where the collective left them: a device result is NOT copied to the host
        # (and the host does not wait for the GPU) until a key is actually looked at; fed back
        # into the next map collective unmodified it never leaves the GPU
        if isinstance(ids, torch.Tensor):
            self._kdev, self._ids_np = ids, None
            self._ev = None
            if ids.is_cuda:
                self._ev = torch.cuda.Event()
                self._ev.record()
        else:
            self._kdev, self._ids_np, self._ev = None, ids, None
        self._n = int(ids.shape[0])
        self._rows = rows
        self._shape = tuple(shape)
        self._keys = None          # key list (lazy)
        self._index = None         # key -> row (lazy)
        self._over = {}            # assigned keys
        self._dead = set()         # deleted base keys

    def pristine(self) -> bool:
        return not self._over and not self._dead

    @property
    def _ids(self) -> np.ndarray:
        if self._ids_np is None:
            if self._ev is not None:
                self._ev.synchronize()           # the producing stream's kernels are done
            self._ids_np = self._kdev.cpu().numpy()
        return self._ids_np

    def _klist(self) -> List:
        if self._keys is None:
            self._keys = self._d.keys_of(self._ids)
        return self._keys

    def _idx(self) -> Dict:
        if self._index is None:
            self._index = dict(zip(self._klist(), range(self._n)))
        return self._index

    def __getitem__(self, k):
        if k in self._over:
            return self._over[k]
        if k in self._dead:
            raise KeyError(k)
        return self._rows[self._idx()[k]].view(self._shape)

    def __setitem__(self, k, v):
        self._over[k] = v
        self._dead.discard(k)

    def __delitem__(self, k):
        if k in self._over:
            del self._over[k]
            if k in self._idx():
                self._dead.add(k)
        elif k in self._idx() and k not in self._dead:
            self._dead.add(k)
        else:
            raise KeyError(k)

    def __contains__(self, k):
        return k in self._over or (k not in self._dead and k in self._idx())

    def __iter__(self):
        base = self._klist()
        if self.pristine():
            yield from base
            return
        for k in base:
            if k not in self._dead and k not in self._over:
                yield k
        yield from self._over

    def __len__(self):
        if self.pristine():
            return self._n
        idx = self._idx()
        return len(idx) - len(self._dead) + sum(1 for k in self._over if k not in idx or k in self._dead)

    def values(self):
        if self.pristine():
            return list(self._rows.view((self._n,) + self._shape).unbind(0))
        return super().values()

    def __repr__(self):
        return f"TensorMap({len(self)} keys, value shape {self._shape}, {self._rows.dtype}, {self._rows.device})"


def _rows_of_one_base(vals: List[torch.Tensor]) -> Optional[torch.Tensor]:
    """Row indices when every value is a whole row of ONE contiguous base tensor (a dict built
    from ``table.unbind(0)`` / ``table[i]``, or from a previous result's rows), else None.
    ``torch.stack`` of n CUDA tensors costs n/128 launches (1563 for 200k values, 56 ms on the
    box, profiles/r2/map_api_*); these checks are four C-level passes and the gather ONE launch.
    A value is row k exactly when it is contiguous, has the base's row numel and starts at k * D."""
    b = vals[0]._base
    if b is None or not b.is_contiguous() or b.dim() < 1 or b.shape[0] == 0:
        return None
    d = b.numel() // b.shape[0]
    if d == 0 or not all(x._base is b for x in vals):
        return None
    n = len(vals)
    if not (all(map(d.__eq__, map(torch.Tensor.numel, vals))) and all(map(torch.Tensor.is_contiguous, vals))):
        return None
    offs = np.fromiter(map(torch.Tensor.storage_offset, vals), dtype=np.int64, count=n) - b.storage_offset()
    if (offs % d).any():
        return None
    return torch.from_numpy(offs // d)


def _stack_rows(vals: List[torch.Tensor]) -> torch.Tensor:
    """[n, numel] rows of n same-shaped tensors: one row gather when they are rows of one base
    tensor, else ONE stack (no per-value reshape views)."""
    if len(vals) > 1024 and vals[0].is_cuda:        # (on the CPU, stack is a memcpy per value)
        idx = _rows_of_one_base(vals)
        if idx is not None:
            b = vals[0]._base
            return b.reshape(b.shape[0], -1).index_select(0, idx.to(b.device))
    v = torch.stack(vals)
    return v.view(len(vals), -1)


def _pack_native(d: "KeyDictionary", mapData):
    """The native one-walk form of :func:`_map_tensors`'s lookup + row checks
    (csrc/pyext/map_ext.cpp): ``(ids, n_missing, rows or None, base)``, or None when the
    extension is not built or the map is not a plain non-empty dict of tensors."""
    if type(mapData) is not dict or not mapData:
        return None
    from ..ops import native
    ext = native.map_ext()
    if ext is None:
        return None
    first = next(iter(mapData.values()))
    if not isinstance(first, torch.Tensor):
        return None
    b = first._base
    base = b if b is not None and b.is_contiguous() else None
    # the same dict passed again unmodified (equal PEP 509 version tag): its walk still holds
    ver = ext.dict_version(mapData)
    c = d._walk_cache
    if c is not None and c[0] == ver and c[1] is mapData and c[2] is base:
        return c[3].copy(), 0, (c[4].copy() if c[4] is not None else None), base
    n = len(mapData)
    ids = np.empty(n, dtype=np.int64)
    rows = np.empty(n, dtype=np.int64)
    # position hint: a fresh dict built from the same key objects as the last complete walk
    # takes those ids by pointer compare instead of a dictionary probe per key
    hint = d._hint if _KEY_HINT else None
    nmiss, rows_ok, _, keys_t = ext.pack(mapData, d.key2id, base, ids, rows, hint[0] if hint else None,
                                         hint[1] if hint else None, _KEY_HINT)
    if _KEY_HINT and not nmiss:
        d._hint = (keys_t, ids.copy())
    rows = rows if rows_ok else None
    # cache only complete walks (every key numbered; ids never change once given)
    d._walk_cache = (ver, mapData, base, ids.copy(), rows.copy() if rows is not None else None, {}) \
        if not nmiss and _WALK_CACHE else None
    return ids, int(nmiss), rows, base


_WALK_CACHE = os.environ.get("MP4X_MAP_WALK_CACHE", "1") == "1"
_KEY_HINT = os.environ.get("MP4X_MAP_KEY_HINT", "1") == "1"


def _take_rows(table: torch.Tensor, rows: np.ndarray) -> torch.Tensor:
    """``table[rows]`` as a fresh tensor: ONE K3 row-gather launch on the GPU; numpy's take on the
    CPU (torch's multi-threaded CPU index_select measured 30-70 ms for 20k x 64 f32 rows on an
    8-CPU container, np.take 0.7 ms)."""
    if table.is_cuda:                               # K3 row gather (5.2 TB/s; index_select ~2.2)
        from ..ops.device_ops import gather_rows   # rows are in range: the native walk checked them
        return gather_rows(table.contiguous(), torch.from_numpy(rows).to(table.device))
    if not table.requires_grad:
        try:
            return torch.from_numpy(np.take(table.numpy(), rows, axis=0))
        except TypeError:                           # no numpy dtype (bf16 ...)
            pass
    return table.index_select(0, torch.from_numpy(rows))


def _map_tensors_packed(engine, d: "KeyDictionary", mapData: Dict, ids_np, nmiss, rows, base):
    """:func:`_map_tensors` after the native walk: misses numbered in one sync round, values
    gathered as rows of their base tensor with ONE index_select (CPU or GPU) when every value is
    a whole row of it (``base`` viewed as [-1, value numel]), else one stack."""
    if getattr(engine, "_keys_presynced", False) or not nmiss:
        _sync_new_keys(engine, [])
        if nmiss:                                   # presynced but a key has no id: a caller bug
            raise KeyError(list(mapData.keys())[int(np.flatnonzero(ids_np < 0)[0])])
    else:
        keys = list(mapData.keys())
        miss = np.flatnonzero(ids_np < 0)
        mk = [keys[i] for i in miss]
        _sync_new_keys(engine, list(dict.fromkeys(mk)))
        ids_np[miss] = d.id_array(mk)
    first = next(iter(mapData.values()))
    shape = tuple(first.shape)
    # the walk cache's entry for this very dict state (if any) also keeps the ids / row indices
    # already on the device: the same dict passed again costs no host->device copies either
    c = d._walk_cache
    dev_cache = None
    if c is not None and c[1] is mapData and c[2] is base and not nmiss:
        from ..ops import native
        if c[0] == native.map_ext().dict_version(mapData):
            dev_cache = c[5]
    dev = first.device
    if rows is not None:
        table = base.reshape(-1, first.numel())
        if dev_cache is not None and table.is_cuda:
            if "rows" not in dev_cache:
                dev_cache["rows"] = torch.from_numpy(rows).to(dev)
            from ..ops.device_ops import gather_rows
            v = gather_rows(table.contiguous(), dev_cache["rows"])
        else:
            v = _take_rows(table, rows)
    else:                                           # (the walk already ruled out one base)
        v = torch.stack(list(mapData.values())).view(len(ids_np), -1)
    if dev_cache is not None and v.is_cuda:
        if "ids" not in dev_cache:
            dev_cache["ids"] = torch.from_numpy(ids_np).to(v.device)
        return dev_cache["ids"], v, shape
    return torch.from_numpy(ids_np).to(v.device), v, shape


def _map_tensors(engine, mapData: Dict):
    """Dict[str, Tensor] -> (ids int64[n], rows [n, numel], value shape); syncs new keys.
    Vectorised: ids through one ``np.fromiter`` + one host->device copy, values through one
    ``torch.stack`` (r1 built a Python list of ids and a reshaped view per value)."""
    d = _dictionary(engine)
    meta, engine._map_meta = getattr(engine, "_map_meta", None), None   # (value shape, dtype) of the round
    if isinstance(mapData, TensorMap) and mapData.pristine() and mapData._d is d:
        _sync_new_keys(engine, [])          # every key is numbered already (collective round)
        rows = mapData._rows.view(mapData._n, -1)
        if mapData._kdev is not None and mapData._kdev.device == rows.device:
            return mapData._kdev, rows, mapData._shape        # ids never left the GPU
        return torch.from_numpy(mapData._ids).to(rows.device), rows, mapData._shape
    pre = getattr(engine, "_prepacked", None)
    engine._prepacked = None
    if pre is not None and pre[0] is mapData and getattr(engine, "_keys_presynced", False):
        ids, nmiss, rows, base = pre[1]           # walked by the agreement round (process_comm)
        if nmiss:                                 # numbered by that round since
            miss = np.flatnonzero(ids < 0)
            keys = list(mapData.keys())
            ids[miss] = d.id_array([keys[i] for i in miss])
        return _map_tensors_packed(engine, d, mapData, ids, 0, rows, base)
    packed = _pack_native(d, mapData)
    if packed is not None:
        return _map_tensors_packed(engine, d, mapData, *packed)
    keys = list(mapData.keys())
    if getattr(engine, "_keys_presynced", False):   # the agreement round numbered them already
        _sync_new_keys(engine, [])
        ids_np = d.id_array(keys)
    else:                                           # ONE lookup pass finds the ids and the misses
        ids_np = d.lookup(keys)
        miss = np.flatnonzero(ids_np < 0)
        mk = [keys[i] for i in miss]
        _sync_new_keys(engine, list(dict.fromkeys(mk)))
        if mk:
            ids_np[miss] = d.id_array(mk)
    vals = list(mapData.values())
    dev = vals[0].device if vals else engine.device
    if vals:
        v = _stack_rows(vals)
        shape = tuple(vals[0].shape)
    elif meta is not None:                          # the agreement round said what the rows are
        shape = tuple(meta[0])
        width = 1
        for x in shape:
            width *= x
        v = torch.empty((0, width), dtype=getattr(torch, meta[1]), device=dev)
    else:
        v = torch.empty((0, 1), device=dev)
        shape = (1,)
    ids = torch.from_numpy(ids_np).to(dev, non_blocking=False)
    return ids, v, shape


def _tensors_map(engine, k: torch.Tensor, v: torch.Tensor, shape) -> "TensorMap":
    return TensorMap(_dictionary(engine), k, v, shape)


def allreduce_map_device(engine, mapData: Dict, operator) -> Dict:
    """``allreduceMap`` for ``Dict[str, torch.Tensor]`` values on the GPU."""
    k, v, shape = _map_tensors(engine, mapData)
    rk, rv = allreduce_sparse(engine, k, v, operator, _dictionary(engine).bits)
    return _tensors_map(engine, rk, rv, shape)


def reduce_map_device(engine, mapData: Dict, operator, root: int) -> Dict:
    """``reduceMap``: the op-reduced union at ``root`` (non-root: its owned share)."""
    k, v, shape = _map_tensors(engine, mapData)
    rk, rv = reduce_sparse(engine, k, v, operator, root, _dictionary(engine).bits)
    return _tensors_map(engine, rk, rv, shape)


def gather_map_device(engine, mapData: Dict, root: int) -> Dict:
    """``gatherMap``: union at root, duplicate keys keep the lowest rank's value (K8)."""
    k, v, shape = _map_tensors(engine, mapData)
    gk, gv = gather_sparse(engine, k, v, root, _dictionary(engine).bits)
    return _tensors_map(engine, gk, gv, shape) if engine.rank == root else mapData


def allgather_map_device(engine, mapData: Dict) -> List[Dict]:
    """``allgatherMap``: every rank's map, indexed by rank."""
    k, v, shape = _map_tensors(engine, mapData)
    ak, av, sizes = allgather_sparse(engine, k, v)
    out, off = [], 0
    for n in sizes:
        out.append(_tensors_map(engine, ak[off:off + n], av[off:off + n], shape))
        off += n
    return out


def _maps_by_dest(engine, maps: List[Dict]):
    """A list of p maps (map j -> rank j) as per-dest (ids, rows) + counts + value shape; ONE
    dictionary sync for all of them."""
    d = _dictionary(engine)
    _sync_new_keys(engine, d.unknown(k for m in maps for k in m.keys()))
    ks, vs, counts, shape = [], [], [], None
    for m in maps:
        packed = _pack_native(d, m)
        if packed is not None:                      # native walk: ids + rows of one base
            ids, _, rows, base = packed
            first = next(iter(m.values()))
            shape = tuple(first.shape)
            dev = first.device
            v = (_take_rows(base.reshape(-1, first.numel()), rows)
                 if rows is not None else torch.stack(list(m.values())).view(len(ids), -1))
            ks.append(torch.from_numpy(ids).to(dev))
            vs.append(v)
            counts.append(len(ids))
            continue
        ids = d.id_array(list(m.keys()))
        vals = list(m.values())
        dev = vals[0].device if vals else engine.device
        if vals:
            shape = tuple(vals[0].shape)
            v = _stack_rows(vals)
        else:
            v = torch.empty((0, 1), device=dev)
        ks.append(torch.from_numpy(ids).to(dev))
        vs.append(v)
        counts.append(len(ids))
    return ks, vs, counts, shape


def reduce_scatter_map_device(engine, mapDataList: List[Dict], operator) -> Dict:
    """``reduceScatterMap``: rank i gets the op-reduction of every rank's ``mapDataList[i]``.
    One ragged all-to-all by explicit destination, then K5 reduce-by-key in rank order."""
    ks, vs, counts, shape = _maps_by_dest(engine, mapDataList)
    shape = engine.all_gather_object(shape)
    shape = next((x for x in shape if x is not None), (1,))
    dev = engine.device
    width = 1
    for d in shape:
        width *= d
    vs = [v if v.numel() else torch.empty((0, width), dtype=next((x.dtype for x in vs if x.numel()), torch.float32),
                                          device=dev) for v in vs]
    dt = next((v.dtype for v in vs if v.numel()), vs[0].dtype)
    keys = torch.cat(ks) if ks else torch.empty(0, dtype=torch.int64, device=dev)
    vals = torch.cat([v.to(dt) for v in vs])
    send = torch.tensor(counts, dtype=torch.int64, device=keys.device)
    recv = torch.empty_like(send)
    engine.coll.all_to_all_single(recv, send)
    rc = [int(x) for x in recv.tolist()]
    rk = torch.empty(sum(rc), dtype=torch.int64, device=keys.device)
    engine.coll.all_to_all_single(rk, keys, rc, counts)
    rv = torch.empty((sum(rc), vals.shape[1]), dtype=vals.dtype, device=vals.device)
    engine.coll.all_to_all_single(rv, vals, rc, counts)
    op = operator if getattr(operator, "is_custom", False) else for_dtype(operator, dtype_of_torch(rv.dtype))
    d = _dictionary(engine)
    # dense dictionary ids in [0, len): K5d by direct addressing (stride 1) when the table is small
    # enough for the rows received, else the sort over the ids' bits
    T = len(d.id2key)
    dense = (0, 1, T) if rk.is_cuda and rk.shape[0] and 0 < T <= min(DENSE_FACTOR * rk.shape[0], DENSE_MAX_SLOTS) \
        else None
    uk, uv, _ = _reduce_by_key(rk, rv, op, d.bits, dense)
    return _tensors_map(engine, uk, uv, shape)


def scatter_map_device(engine, mapDataList: Optional[List[Dict]], root: int) -> Dict:
    """``scatterMap``: root's ``mapDataList[i]`` lands at rank i (grouped p2p from the root)."""
    r, p = engine.rank, engine.p
    if r == root:
        ks, vs, counts, shape = _maps_by_dest(engine, mapDataList)
        dt = next((v.dtype for v in vs if v.numel()), torch.float32)
        meta = (counts, shape or (1,), str(dt).replace("torch.", ""))
    else:
        _sync_new_keys(engine, [])        # matches the root's one dictionary sync
        meta = None
    counts, shape, dt = engine.all_gather_object(meta)[root]
    width = 1
    for d in shape:
        width *= d
    dev = engine.device
    if r == root:
        sends = []
        for j in range(p):
            if j != root and counts[j]:
                sends += [(ks[j], j), (vs[j].reshape(counts[j], width).to(getattr(torch, dt)).contiguous(), j)]
        engine.coll.p2p(sends, [])
        return _tensors_map(engine, ks[root], vs[root].reshape(counts[root], width), shape)
    k = torch.empty(counts[r], dtype=torch.int64, device=dev)
    v = torch.empty((counts[r], width), dtype=getattr(torch, dt), device=dev)
    if counts[r]:
        engine.coll.p2p([], [(k, root), (v, root)])
    return _tensors_map(engine, k, v, shape)


def broadcast_map_device(engine, mapData: Dict, root: int) -> Dict:
    """``broadcastMap``: root's map on every rank."""
    if engine.rank == root:
        k, v, shape = _map_tensors(engine, mapData)
    else:
        _sync_new_keys(engine, [])
        k = v = None
    bk, bv = broadcast_sparse(engine, k, v, root)
    shape = engine.all_gather_object(shape if engine.rank == root else None)[root]
    return _tensors_map(engine, bk, bv, shape)
