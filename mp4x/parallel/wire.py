"""Message layout of the host data plane.

Equivalent of the reference's ``ArrayMetaData`` / ``MapMetaData`` headers and
per-type Kryo serializers (J/meta/ArrayMetaData.java:103-133,
J/meta/MapMetaData.java:117-143, J/operand/DoubleOperand.java:53-258), but
laid out for zero-copy numpy I/O::

    u32 meta_len | msgpack(meta) | blob_0 | blob_1 | ...

``meta["s"]`` lists the segments ``[rank, from, to, nbytes]`` (ARRAY) or the
maps ``[rank, keys_nbytes, vals_nbytes, vkind, dim]`` (MAP).  Primitive blobs
are the raw little-endian element bytes; object/string blobs come from the
operand's serializer.  ``compress`` applies zlib (the reference's Deflate
wrapper) per blob.
"""
from __future__ import annotations

import struct
import zlib
from typing import Dict, List, Sequence, Tuple

import msgpack
import numpy as np

from ..operands import Operand

_U32 = struct.Struct("<I")
ZLEVEL = 1


def _z(b, compress: bool):
    return zlib.compress(bytes(b), ZLEVEL) if compress else b


def _unz(b, compress: bool):
    return zlib.decompress(b) if compress else b


def _finish(meta: dict, blobs: List) -> List:
    m = msgpack.packb(meta, use_bin_type=True)
    return [_U32.pack(len(m)), m] + blobs


def _split(body) -> Tuple[dict, memoryview]:
    mv = memoryview(body)
    (ml,) = _U32.unpack(mv[:4])
    meta = msgpack.unpackb(mv[4:4 + ml], raw=False, strict_map_key=False)
    return meta, mv[4 + ml:]


# ------------------------------------------------------------------ ARRAY
def pack_segments(arr, segs: Sequence[Tuple[int, int, int]], operand: Operand) -> List:
    """segs = [(rank, from, to)] of ``arr`` (numpy array or Python list)."""
    comp = operand.compress
    blobs = []
    seg_meta = []
    for (rk, f, t) in segs:
        if operand.is_primitive:
            b = arr[f:t]
            if not b.flags.c_contiguous:
                b = np.ascontiguousarray(b)
            b = _z(memoryview(b).cast("B"), comp) if comp else memoryview(b).cast("B")
        else:
            b = _z(operand.serializer.write_list(arr[f:t]), comp)
        blobs.append(b)
        seg_meta.append([int(rk), int(f), int(t), len(b)])
    return _finish({"s": seg_meta, "z": comp}, blobs)


def unpack_segments(body, operand: Operand):
    """Yields (rank, from, to, data) with data a numpy view / list of objects."""
    meta, rest = _split(body)
    comp = meta["z"]
    off = 0
    out = []
    for rk, f, t, nb in meta["s"]:
        raw = rest[off:off + nb]
        off += nb
        if operand.is_primitive:
            raw = _unz(raw, comp)
            data = np.frombuffer(raw, dtype=operand.np_dtype, count=t - f)
        else:
            data = operand.serializer.read_list(_unz(raw, comp))
        out.append((rk, f, t, data))
    return out


# ------------------------------------------------------------------ MAP
VK_SCALAR, VK_VEC, VK_OBJ = 0, 1, 2

_SEP = "\0"


def encode_keys(keys) -> bytes:
    """Wire form of a key list for the peer-to-peer key rounds.  ``S`` + the UTF-8 of the keys
    joined by NUL when every key is a ``str`` without NUL (the reference's keys are Strings:
    one C-level join / split, ~10 ms for 200k keys); ``E`` = no keys; otherwise ``P`` + pickle
    (any hashable keys, between this job's own ranks)."""
    keys = keys if isinstance(keys, list) else list(keys)
    if not keys:
        return b"E"
    try:
        j = _SEP.join(keys)            # C-level; TypeError as soon as a key is not a str
    except TypeError:
        j = None
    if j is not None and j.count(_SEP) == len(keys) - 1:
        return b"S" + j.encode("utf-8", "surrogatepass")
    import pickle
    return b"P" + pickle.dumps(keys, protocol=pickle.HIGHEST_PROTOCOL)


def decode_keys(blob: bytes) -> List:
    tag = blob[:1]
    if tag == b"E" or not blob:
        return []
    if tag == b"S":
        return blob[1:].decode("utf-8", "surrogatepass").split(_SEP)
    if tag == b"P":
        import pickle
        return pickle.loads(blob[1:])
    raise ValueError(f"bad key block tag {tag!r}")



def stack_rows(vals: List, dtype=None) -> np.ndarray:
    """``np.stack(vals).astype(dtype, copy=False)`` for equal-shaped numpy rows — one native copy
    per row (csrc/pyext/hostmap_ext.cpp ``stack_rows``) when they all share the dtype."""
    v0 = vals[0]
    dt = np.dtype(dtype) if dtype is not None else v0.dtype
    if isinstance(vals, list) and isinstance(v0, np.ndarray) and v0.dtype == dt and v0.size:
        from ..ops import native
        ext = native.hostmap_ext()
        if ext is not None:
            out = np.empty((len(vals),) + v0.shape, dtype=dt)
            if ext.stack_rows(vals, out):
                return out
    return np.stack(vals).astype(dt, copy=False)


def _stack_like(vals: np.ndarray, rows: List):
    """``rows`` stacked as a fresh [len(rows), dim] array of ``vals``' dtype, or None unless every
    row is a 1-D-equivalent numpy row of exactly that dtype and size (the native copy checks each
    row's buffer format and length in C; without the extension, the same checks in Python)."""
    out = np.empty((len(rows),) + vals.shape[1:], dtype=vals.dtype)
    from ..ops import native
    ext = native.hostmap_ext()
    if ext is not None:
        return out if ext.stack_rows(rows, out) else None
    if all(isinstance(r, np.ndarray) and r.dtype == vals.dtype and r.shape == vals.shape[1:] for r in rows):
        return np.stack(rows)
    return None


def _encode_map(d: Dict, operand: Operand):
    keys = list(d.keys())
    kb = msgpack.packb(keys, use_bin_type=True)
    vals = list(d.values())
    if operand.is_primitive:
        if vals and isinstance(vals[0], np.ndarray):
            dim = int(vals[0].size)
            vb = np.ascontiguousarray(stack_rows(vals, operand.np_dtype)).tobytes()
            return kb, vb, VK_VEC, dim
        vb = np.asarray(vals, dtype=operand.np_dtype).tobytes()
        return kb, vb, VK_SCALAR, 1
    return kb, operand.serializer.write_list(vals), VK_OBJ, 0


def pack_maps(maps: Sequence[Tuple[int, Dict]], operand: Operand) -> List:
    comp = operand.compress
    blobs = []
    mm = []
    for rk, d in maps:
        kb, vb, vk, dim = _encode_map(d, operand)
        kb, vb = _z(kb, comp), _z(vb, comp)
        blobs += [kb, vb]
        mm.append([int(rk), len(kb), len(vb), vk, dim])
    return _finish({"m": mm, "z": comp}, blobs)


def unpack_maps(body, operand: Operand, raw_values: bool = False):
    """Returns [(rank, keys, values)] where values is an ndarray (scalar: 1-D, vec: 2-D) or list."""
    meta, rest = _split(body)
    comp = meta["z"]
    off = 0
    out = []
    for rk, kn, vn, vk, dim in meta["m"]:
        kb = _unz(rest[off:off + kn], comp)
        off += kn
        vb = _unz(rest[off:off + vn], comp)
        off += vn
        keys = msgpack.unpackb(kb, raw=False)
        if vk == VK_SCALAR:
            vals = np.frombuffer(vb, dtype=operand.np_dtype, count=len(keys)).copy()
        elif vk == VK_VEC:
            vals = np.frombuffer(vb, dtype=operand.np_dtype).copy().reshape(len(keys), dim)
        else:
            vals = operand.serializer.read_list(vb)
        out.append((rk, keys, vals))
    return out


def to_dict(keys, vals, vkind_vec: bool = None) -> Dict:
    if isinstance(vals, np.ndarray):
        if vals.ndim == 2:
            return dict(zip(keys, list(vals)))
        return dict(zip(keys, vals.tolist()))
    return dict(zip(keys, vals))


def merge_reduce(local: Dict, keys, vals, op) -> Dict:
    """local[k] = op(local[k], v) for shared keys, insert new keys (MapReduce deserializer,
    J/operand/DoubleOperand.java:225-257) — vectorised over the shared keys."""
    if isinstance(vals, np.ndarray) and vals.ndim == 1 and not op.is_custom:
        shared_i = [i for i, k in enumerate(keys) if k in local]
        if shared_i:
            sk = [keys[i] for i in shared_i]
            acc = np.array([local[k] for k in sk], dtype=vals.dtype)
            with np.errstate(over="ignore", invalid="ignore"):
                op.reduce_into(acc, vals[shared_i])
            for k, v in zip(sk, acc.tolist()):
                local[k] = v
        if len(shared_i) != len(keys):
            vl = vals.tolist()
            for k, v in zip(keys, vl):
                if k not in local:
                    local[k] = v
        return local
    if isinstance(vals, np.ndarray) and vals.ndim == 2 and not op.is_custom:
        # vectorised over the shared keys: ONE stack of the local rows, ONE reduce, row views back
        cur = list(map(local.get, keys))
        shared_i = [i for i, c in enumerate(cur) if c is not None]
        acc = _stack_like(vals, [cur[i] for i in shared_i]) if shared_i else vals[:0]
        if acc is not None:
            if shared_i:
                with np.errstate(over="ignore", invalid="ignore"):
                    op.reduce_into(acc, vals[shared_i])
                for i, row in zip(shared_i, acc):
                    local[keys[i]] = row
            if len(shared_i) != len(keys):
                for k, c, row in zip(keys, cur, vals):
                    if c is None:
                        local[k] = row
            return local
    if isinstance(vals, np.ndarray) and vals.ndim == 2:
        for k, row in zip(keys, vals):
            cur = local.get(k)
            if cur is None:
                local[k] = row
            else:
                cur = np.array(cur, copy=True)
                with np.errstate(over="ignore", invalid="ignore"):
                    op.reduce_into(cur, row)
                local[k] = cur
        return local
    for k, v in zip(keys, vals):
        if k in local:
            local[k] = op.apply(local[k], v)
        else:
            local[k] = v
    return local
