"""Columnar host ``allreduceMap`` for primitive values (``Map<String, double>`` counts and
``Map<String, float[]>`` rows on the CPU).

Reference: ``ProcessCommSlave.allreduceMap`` (J/comm/ProcessCommSlave.java:2053-2088) = owner
partition by ``key.hashCode() % p`` -> reduce-scatter of per-owner maps -> allgather -> merge,
with the MapReduce deserialiser folding each received value into the local map
(J/operand/DoubleOperand.java:225-257).

Here a map travels as two columns — its keys (one NUL-joined UTF-8 blob) and its values (one
``[n, dim]`` array) — and is never rebuilt entry by entry in between:

* partition: one native pass computes every key's owner (``owner_ids``), one stable argsort
  splits keys and rows;
* reduce-scatter (direct: each block straight to its owner, p-1 concurrent sends): the owner
  concatenates its own block and the p-1 received ones in RANK order and reduces equal keys
  vectorised — first-occurrence ids through one C-level ``dict.setdefault`` map, a stable sort,
  one ``ufunc.reduceat`` (a left fold in rank order: deterministic, like the reference's ring
  fold);
* allgather (direct): every owner's (keys, rows) block to every rank; the result is the
  concatenation (owners are disjoint).

The result of a vector map is a :class:`RowMap` (a ``MutableMapping`` over the columns, rows as
views; passing it to the next collective skips the per-entry walk entirely); a scalar map
returns a plain ``dict`` of Python scalars as before.
"""
from __future__ import annotations

import struct
import zlib
from collections.abc import ItemsView, MutableMapping, ValuesView
from typing import List, Optional, Sequence, Tuple

import numpy as np

from ..operands import Operand
from ..operators import OpCode
from .wire import decode_keys, encode_keys, stack_rows

_HDR = struct.Struct("<qqqqb?")     # nkeys, key bytes, row bytes, dim (-1: scalar, -2: unknown), has-rows, z
_UFUNC = {OpCode.SUM: np.add, OpCode.MAX: np.maximum, OpCode.MIN: np.minimum, OpCode.PROD: np.multiply,
          OpCode.BAND: np.bitwise_and, OpCode.BOR: np.bitwise_or, OpCode.BXOR: np.bitwise_xor}


class RowMap(MutableMapping):
    """``Dict[key, ndarray row]`` over two columns: a key list and one ``[n, dim]`` array
    (``rows[i]`` is ``keys[i]``'s value, a view).  ``len``, iteration, ``items()`` and the next
    collective read the columns directly; the key -> row index (one dict of n entries) is
    built on the first lookup (``index_built`` tells whether it exists yet).  The first
    structural change (insert / delete / replacing a value) turns it into a plain dict
    internally, so it behaves exactly like the dict the reference returns.  Keys are unique by
    construction (disjoint owners)."""

    __slots__ = ("_keys", "_rows", "_index", "_d")

    def __init__(self, keys: List, rows: np.ndarray):
        self._keys = keys
        self._rows = rows
        self._index: Optional[dict] = None
        self._d: Optional[dict] = None

    @property
    def index_built(self) -> bool:
        return self._index is not None or self._d is not None

    def _idx(self) -> dict:
        if self._index is None:
            self._index = dict(zip(self._keys, range(len(self._keys))))
        return self._index

    def items(self):
        return self._d.items() if self._d is not None else _RowItems(self)

    def values(self):
        return self._d.values() if self._d is not None else _RowValues(self)

    # -- columnar access (the collectives use it to skip the per-entry walk)
    def columns(self) -> Optional[Tuple[List, np.ndarray]]:
        return None if self._d is not None else (self._keys, self._rows)

    def _dict(self) -> dict:
        if self._d is None:
            self._d = dict(zip(self._keys, self._rows))
            self._keys, self._rows, self._index = None, None, None
        return self._d

    def __getitem__(self, k):
        if self._d is not None:
            return self._d[k]
        return self._rows[self._idx()[k]]

    def __setitem__(self, k, v):
        self._dict()[k] = v

    def __delitem__(self, k):
        del self._dict()[k]

    def __contains__(self, k):
        return k in (self._d if self._d is not None else self._idx())

    def __iter__(self):
        return iter(self._d if self._d is not None else self._keys)

    def __len__(self):
        return len(self._d) if self._d is not None else len(self._keys)

    def __repr__(self):
        return f"RowMap({len(self)} keys)"


class _RowItems(ItemsView):
    def __iter__(self):
        m = self._mapping
        return iter(m.items()) if m._d is not None else zip(m._keys, m._rows)


class _RowValues(ValuesView):
    def __iter__(self):
        m = self._mapping
        return iter(m.values()) if m._d is not None else iter(m._rows)


def columns_of(mapData, operand: Operand) -> Tuple[List, Optional[np.ndarray], int]:
    """(keys, values column, dim) of a map; dim -1 = scalar values, -2 = empty map (shape
    unknown on this rank)."""
    if isinstance(mapData, RowMap) and mapData.columns() is not None:
        keys, rows = mapData.columns()
        if rows.dtype != operand.np_dtype:
            rows = rows.astype(operand.np_dtype)
        return list(keys), rows, int(rows.shape[1]) if rows.ndim == 2 else -1
    if not mapData:
        return [], None, -2
    keys = list(mapData.keys())
    vals = list(mapData.values())
    v0 = vals[0]
    if isinstance(v0, np.ndarray) and v0.ndim >= 1:
        rows = stack_rows(vals, operand.np_dtype).reshape(len(vals), -1)
        return keys, rows, int(rows.shape[1])
    if isinstance(v0, (list, tuple)):
        rows = np.asarray(vals, dtype=operand.np_dtype).reshape(len(vals), -1)
        return keys, rows, int(rows.shape[1])
    return keys, np.fromiter(vals, dtype=operand.np_dtype, count=len(vals)), -1


def owners(keys: List, p: int) -> np.ndarray:
    out = np.empty(len(keys), dtype=np.int32)
    from ..ops import native
    ext = native.hostmap_ext()
    if ext is not None and ext.owner_ids(keys, p, out):
        return out
    from ..utils.hashing import owner_of
    return np.fromiter((owner_of(k, p) for k in keys), dtype=np.int32, count=len(keys))


def _pack(keys: Sequence, rows: Optional[np.ndarray], dim: int, compress: bool) -> List:
    kb = encode_keys(keys)
    rb = memoryview(np.ascontiguousarray(rows)).cast("B") if rows is not None and len(keys) else b""
    if compress:
        kb, rb = zlib.compress(kb, 1), zlib.compress(bytes(rb), 1)
    return [_HDR.pack(len(keys), len(kb), len(rb), dim, rows is not None and len(keys) > 0, compress), kb, rb]


def _unpack(body, np_dtype) -> Tuple[List, Optional[np.ndarray], int]:
    n, kn, rn, dim, has_rows, comp = _HDR.unpack_from(body, 0)
    mv = memoryview(body)
    o = _HDR.size
    kb = bytes(mv[o:o + kn])
    rb = mv[o + kn:o + kn + rn]
    if comp:
        kb = zlib.decompress(kb)
        rb = zlib.decompress(rb) if rn else b""
    keys = decode_keys(kb) if n else []
    rows = None
    if has_rows:
        rows = np.frombuffer(rb, dtype=np_dtype, count=n * max(1, dim))
        rows = rows.reshape(n, dim) if dim >= 0 else rows
    return keys, rows, dim


def _group_reduce(keys: List, rows: np.ndarray, op) -> Tuple[List, np.ndarray]:
    """Reduce rows of equal keys, first-occurrence order, rows combined in position order."""
    n = len(keys)
    first = {}
    fo = np.fromiter(map(first.setdefault, keys, range(n)), dtype=np.int64, count=n)
    if len(first) == n:
        return keys, rows
    is_new = fo == np.arange(n)
    gid = (np.cumsum(is_new) - 1)[fo]
    order = np.argsort(gid, kind="stable")
    g_sorted = gid[order]
    starts = np.flatnonzero(np.r_[True, g_sorted[1:] != g_sorted[:-1]])
    uf = _UFUNC[op.code]
    with np.errstate(over="ignore", invalid="ignore"):
        # dtype=: add/multiply reductions of small ints would otherwise widen to int64
        red = uf.reduceat(rows[order], starts, axis=0, dtype=rows.dtype)
    ukeys = list(first.keys())             # insertion order == first occurrence == group id
    return ukeys, red


def supported(operand: Operand, op) -> bool:
    """Rank-independent eligibility (the operand / operator are the same on every rank)."""
    return operand.is_primitive and not getattr(op, "is_custom", False) and op.code in _UFUNC


def allreduce_map(engine, mapData, operand: Operand, op):
    """The columnar allreduceMap over ``engine`` (HostEngine: TCP mesh), direct schedule."""
    p, r = engine.p, engine.rank
    keys, vals, dim = columns_of(mapData, operand)
    comp = bool(operand.compress)
    np_dtype = operand.np_dtype
    # ---- partition by owner
    if keys:
        own = owners(keys, p)
        order = np.argsort(own, kind="stable")
        counts = np.bincount(own, minlength=p)
        bounds = np.r_[0, np.cumsum(counts)]
    # ---- reduce-scatter: block b -> owner b
    tag = engine.next_tag()
    blocks_k: List[List] = [[] for _ in range(p)]
    blocks_v: List[Optional[np.ndarray]] = [None] * p
    if keys:
        karr = np.empty(len(keys), dtype=object)
        karr[:] = keys
        ks = karr[order]
        vs = vals[order]
        for b in range(p):
            lo, hi = bounds[b], bounds[b + 1]
            blocks_k[b] = ks[lo:hi].tolist()
            blocks_v[b] = vs[lo:hi]
    for j in range(1, p):
        b = (r + j) % p
        engine.t.send(b, tag, _pack(blocks_k[b], blocks_v[b], dim, comp))
    mine_k, mine_v = [blocks_k[r]], [blocks_v[r]]
    recv = {}
    for j in range(1, p):
        src = (r - j) % p
        recv[src] = _unpack(engine.t.recv(src, tag), np_dtype)
    dims = {dim} | {d for _, _, d in recv.values()}
    dims.discard(-2)
    if len(dims) > 1:
        raise ValueError(f"allreduceMap: ranks disagree on the value shape ({sorted(dims)})")
    dim_all = dims.pop() if dims else -2
    # rank order: own block at position r
    cat_k: List = []
    cat_v: List[np.ndarray] = []
    for src in range(p):
        k, v = (mine_k[0], mine_v[0]) if src == r else recv[src][:2]
        if k:
            cat_k += k
            cat_v.append(v)
    if cat_k:
        allv = np.concatenate(cat_v, axis=0) if len(cat_v) > 1 else cat_v[0]
        rk, rv = _group_reduce(cat_k, allv, op)
    else:
        rk, rv = [], None
    # ---- allgather of the owned results (direct)
    tag = engine.next_tag()
    body = _pack(rk, rv, dim_all, comp)
    for j in range(1, p):
        engine.t.send((r + j) % p, tag, body)
    parts_k: List = []
    parts_v: List[np.ndarray] = []
    got = {}
    for j in range(1, p):
        src = (r - j) % p
        got[src] = _unpack(engine.t.recv(src, tag), np_dtype)
    for src in range(p):
        k, v = (rk, rv) if src == r else got[src][:2]
        if k:
            parts_k += k
            parts_v.append(v)
    if dim_all == -2 or not parts_k:
        return {}
    allv = np.concatenate(parts_v, axis=0) if len(parts_v) > 1 else np.array(parts_v[0], copy=True)
    if dim_all == -1:
        return dict(zip(parts_k, allv.tolist()))
    return RowMap(parts_k, allv)


__all__ = ["RowMap", "allreduce_map", "supported", "columns_of", "owners"]
