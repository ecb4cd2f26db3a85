"""torch-facing wrappers of the native CDNA4 kernels.

Every wrapper validates shapes, dtypes, devices and contiguity on the host BEFORE the
launch (a bad pointer on a GPU is a machine-wide fault, not an exception) and launches on
the current torch stream.
"""
from __future__ import annotations

import os
from typing import NamedTuple, Optional, Sequence, Tuple

import torch

from ..operators import DType, dtype_of_torch
from . import native
from .native import check, ptr_array, stream_ptr

QBLOCK = 256


def _dev_check(*ts):
    dev = None
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise ValueError("device op needs GPU tensors")
        if not t.is_contiguous():
            raise ValueError("device op needs contiguous tensors")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise ValueError("all tensors must be on one device")


def reduce_(out: torch.Tensor, inputs: Sequence[torch.Tensor], op: int, dtype: Optional[DType] = None,
            stream=None) -> torch.Tensor:
    """out = op(inputs[0], inputs[1], ...) elementwise, in input order (out may alias inputs[0])."""
    if not inputs:
        raise ValueError("no inputs")
    _dev_check(out, *inputs)
    n = out.numel()
    for t in inputs:
        if t.numel() != n or t.dtype != out.dtype:
            raise ValueError(f"reduce_: shape/dtype mismatch {t.shape}/{t.dtype} vs {out.shape}/{out.dtype}")
    dt = dtype if dtype is not None else dtype_of_torch(out.dtype)
    pp, keep = ptr_array([t.data_ptr() for t in inputs])
    check(native.hip().mp4x_reduce(int(dt), int(op), out.data_ptr(), pp, len(inputs), n, stream_ptr(stream)),
          "mp4x_reduce")
    return out


def reduce_strided_(out: torch.Tensor, base: torch.Tensor, nin: int, op: int, stream=None) -> torch.Tensor:
    """out = op over nin equal chunks of ``base`` (laid out back to back, each out.numel() long)."""
    _dev_check(out, base)
    n = out.numel()
    if base.numel() < n * nin or base.dtype != out.dtype:
        raise ValueError("reduce_strided_: base too small or dtype mismatch")
    dt = dtype_of_torch(out.dtype)
    check(native.hip().mp4x_reduce_strided(int(dt), int(op), out.data_ptr(), base.data_ptr(), n, nin, n,
                                           stream_ptr(stream)), "mp4x_reduce_strided")
    return out


def scale_(out: torch.Tensor, inp: torch.Tensor, s: float, stream=None) -> torch.Tensor:
    _dev_check(out, inp)
    if out.numel() != inp.numel() or out.dtype != inp.dtype:
        raise ValueError("scale_: mismatch")
    check(native.hip().mp4x_scale(int(dtype_of_torch(out.dtype)), out.data_ptr(), inp.data_ptr(), float(s),
                                  out.numel(), stream_ptr(stream)), "mp4x_scale")
    return out


def segment_copy_(dst: torch.Tensor, src: torch.Tensor, segs: Sequence[Tuple[int, int, int]], stream=None):
    """segs = [(dst_elem_off, src_elem_off, nelems)] copied in one launch."""
    _dev_check(dst, src)
    if not segs:
        return dst
    es = dst.element_size()
    if src.element_size() != es:
        raise ValueError("segment_copy_: element size mismatch")
    dn, sn = dst.numel(), src.numel()
    for d, s, l in segs:
        if d < 0 or s < 0 or l < 0 or d + l > dn or s + l > sn:
            raise ValueError(f"segment_copy_: segment {(d, s, l)} out of bounds ({dn}, {sn})")
    segs = [x for x in segs if x[2] > 0]
    if not segs:
        return dst
    table = torch.tensor([d * es for d, _, _ in segs] + [s * es for _, s, _ in segs] + [l * es for _, _, l in segs],
                         dtype=torch.int64).pin_memory().to(dst.device, non_blocking=True)
    max_len = max(l for _, _, l in segs) * es
    check(native.hip().mp4x_segment_copy(dst.data_ptr(), src.data_ptr(), table.data_ptr(), len(segs), max_len,
                                         stream_ptr(stream)), "mp4x_segment_copy")
    # `table` may be freed right away: the caching allocator only reuses it in stream order
    return dst


def gather_rows(inp: torch.Tensor, idx: torch.Tensor, out: Optional[torch.Tensor] = None, stream=None):
    """out[i] = inp[idx[i]] for a 2-D (rows, ...) tensor."""
    _dev_check(inp, idx)
    if idx.dtype != torch.int64:
        raise ValueError("gather_rows: idx must be int64")
    rows = inp.shape[0]
    row_bytes = inp[0].numel() * inp.element_size() if rows else 0
    if out is None:
        out = torch.empty((idx.numel(),) + tuple(inp.shape[1:]), dtype=inp.dtype, device=inp.device)
    _dev_check(out)
    check(native.hip().mp4x_gather_rows(out.data_ptr(), inp.data_ptr(), idx.data_ptr(), idx.numel(), row_bytes,
                                        stream_ptr(stream)), "mp4x_gather_rows")
    return out


# ------------------------------------------------------------------ fp8 codec (K6)
def quant_fp8(x: torch.Tensor, q: Optional[torch.Tensor] = None, scales: Optional[torch.Tensor] = None,
              stream=None):
    """Block-scaled e4m3 quantisation (256 elements / scale). Returns (q uint8[n], scales f32[nblk])."""
    _dev_check(x)
    n = x.numel()
    if n % 4:
        raise ValueError("quant_fp8: n must be a multiple of 4")
    nblk = (n + QBLOCK - 1) // QBLOCK
    if q is None:
        q = torch.empty(n, dtype=torch.uint8, device=x.device)
    if scales is None:
        scales = torch.empty(nblk, dtype=torch.float32, device=x.device)
    if q.numel() < n or scales.numel() < nblk:
        raise ValueError("quant_fp8: output too small")
    check(native.hip().mp4x_quant_fp8(int(dtype_of_torch(x.dtype)), x.data_ptr(), n, q.data_ptr(), scales.data_ptr(),
                                      stream_ptr(stream)), "mp4x_quant_fp8")
    return q, scales


def dequant_reduce_fp8(out: Optional[torch.Tensor], qs: Sequence[torch.Tensor], ss: Sequence[torch.Tensor], n: int,
                       accumulate: bool = False, q_out: Optional[torch.Tensor] = None,
                       s_out: Optional[torch.Tensor] = None, out_dtype=None, stream=None):
    nblk = (n + QBLOCK - 1) // QBLOCK
    for q, s in zip(qs, ss):
        _dev_check(q, s)
        if q.numel() < n or s.numel() < nblk:
            raise ValueError("dequant_reduce_fp8: input too small")
    if out is not None:
        _dev_check(out)
        if out.numel() < n:
            raise ValueError("dequant_reduce_fp8: out too small")
        dt = dtype_of_torch(out.dtype)
    else:
        dt = dtype_of_torch(out_dtype or torch.float32)
    if q_out is not None and (q_out.numel() < n or s_out is None or s_out.numel() < nblk):
        raise ValueError("dequant_reduce_fp8: requant outputs too small")
    lib = native.hip()
    done = 0
    first = True
    while done < len(qs):
        k = min(8, len(qs) - done)
        qp, k1 = ptr_array([t.data_ptr() for t in qs[done:done + k]])
        sp, k2 = ptr_array([t.data_ptr() for t in ss[done:done + k]])
        last = done + k == len(qs)
        check(lib.mp4x_dequant_reduce_fp8(int(dt), out.data_ptr() if out is not None else None, qp, sp, k, n,
                                          int(accumulate or not first),
                                          q_out.data_ptr() if (q_out is not None and last) else None,
                                          s_out.data_ptr() if (s_out is not None and last) else None,
                                          stream_ptr(stream)), "mp4x_dequant_reduce_fp8")
        done += k
        first = False
    return out


def dequant_fp8(q: torch.Tensor, scales: torch.Tensor, n: int, out: torch.Tensor, stream=None):
    return dequant_reduce_fp8(out, [q], [scales], n, stream=stream)


# ------------------------------------------------------------------ sparse (K4/K5/K7)
def key_owner(keys: torch.Tensor, p: int, stream=None):
    _dev_check(keys)
    n = keys.numel()
    dest = torch.empty(n, dtype=torch.int32, device=keys.device)
    hist = torch.zeros(p, dtype=torch.int32, device=keys.device)
    check(native.hip().mp4x_key_owner(keys.data_ptr(), n, p, dest.data_ptr(), hist.data_ptr(), stream_ptr(stream)),
          "mp4x_key_owner")
    return dest, hist


ZS_BLOCK = 256
ZS_MAX_CHUNKS = 256      # the chunk table is staged in LDS


def _zs_table(chunks, dev):
    starts = [int(c[0]) for c in chunks]
    lens = [int(c[1]) for c in chunks]
    bs = [0]
    for ln in lens:
        bs.append(bs[-1] + (ln + ZS_BLOCK - 1) // ZS_BLOCK)
    return torch.tensor(starts + lens + bs, dtype=torch.int64, device=dev), bs


def zs_encode(x: torch.Tensor, chunks=None, stream=None):
    """K6b lossless zero suppression of a flat tensor, per chunk ``(start, len)`` (default: whole).

    Returns ``(masks int64[4*nblk], counts int32[nblk], vals x.dtype[nnz], nnz per chunk, blk_start)``;
    chunk j owns blocks ``blk_start[j]:blk_start[j+1]`` and its non-zero words are the j-th
    consecutive run of ``vals``.  One device->host read (the per-chunk totals)."""
    _dev_check(x)
    x = x.reshape(-1)
    if chunks is None:
        chunks = [(0, x.numel())]
    if len(chunks) > ZS_MAX_CHUNKS:
        raise ValueError(f"zs_encode: at most {ZS_MAX_CHUNKS} chunks per call")
    dev = x.device
    table, bs = _zs_table(chunks, dev)
    nblk = bs[-1]
    total = sum(int(c[1]) for c in chunks)
    masks = torch.empty(4 * nblk, dtype=torch.int64, device=dev)
    counts = torch.empty(nblk, dtype=torch.int32, device=dev)
    offs = torch.zeros(nblk + 1, dtype=torch.int64, device=dev)
    vals = torch.empty(max(total, 1), dtype=x.dtype, device=dev)
    lib = native.hip()
    tb = lib.mp4x_zs_temp_bytes(nblk)
    temp = torch.empty(max(tb, 1), dtype=torch.uint8, device=dev)
    check(lib.mp4x_zs_encode(x.element_size(), x.data_ptr(), table.data_ptr(), len(chunks), nblk, masks.data_ptr(),
                             counts.data_ptr(), offs.data_ptr(), vals.data_ptr(), temp.data_ptr(), tb,
                             stream_ptr(stream)), "mp4x_zs_encode")
    at = offs[torch.tensor(bs, dtype=torch.int64, device=dev)].tolist() if nblk else [0] * len(bs)
    nnz = [at[j + 1] - at[j] for j in range(len(chunks))]
    return masks, counts, vals[:at[-1]], nnz, bs


def zs_decode(masks: torch.Tensor, counts: torch.Tensor, vals: torch.Tensor, chunks, out: torch.Tensor,
              stream=None):
    """Inverse of :func:`zs_encode`: chunk j (masks / counts / vals concatenated in chunk order)
    expands into ``out.view(-1)[start_j : start_j + len_j]``."""
    _dev_check(masks, counts, vals, out)
    if len(chunks) > ZS_MAX_CHUNKS:
        raise ValueError(f"zs_decode: at most {ZS_MAX_CHUNKS} chunks per call")
    dev = out.device
    table, bs = _zs_table(chunks, dev)
    nblk = bs[-1]
    if nblk == 0:
        return out
    if masks.numel() != 4 * nblk or counts.numel() != nblk:
        raise ValueError("zs_decode: masks / counts do not match the chunk table")
    if vals.element_size() != out.element_size():
        raise ValueError("zs_decode: vals / out word size differ")
    offs = torch.empty(nblk + 1, dtype=torch.int64, device=dev)
    lib = native.hip()
    tb = lib.mp4x_zs_temp_bytes(nblk)
    temp = torch.empty(max(tb, 1), dtype=torch.uint8, device=dev)
    check(lib.mp4x_zs_decode(out.element_size(), masks.data_ptr(), counts.data_ptr(),
                             vals.data_ptr() if vals.numel() else None, table.data_ptr(), len(chunks), nblk,
                             out.data_ptr(), offs.data_ptr(), temp.data_ptr(), tb, stream_ptr(stream)),
          "mp4x_zs_decode")
    return out


PACK_MAX_P = 2048


def partition_pack(keys: torch.Tensor, vals: Optional[torch.Tensor], p: int, want_perm: bool = False,
                   want_range: bool = False, stream=None):
    """Fused K4b stable partition by owner ``(uint64)key % p``.

    Returns ``(out_keys, out_vals, counts int64[p], perm)``; ``out_vals`` is None when
    ``vals`` is None, ``perm`` (source row of each slot) only with ``want_perm``.  Rows whose
    size is not a multiple of 16 bytes are packed with :func:`gather_rows` through ``perm``.
    ``want_range``: ``counts`` has two more entries, the smallest and largest key (0, 0 when
    empty), reduced inside the same kernels.
    """
    _dev_check(keys, vals)
    if keys.dtype != torch.int64:
        raise ValueError("partition_pack: keys must be int64")
    if not 1 <= p <= PACK_MAX_P:
        raise ValueError(f"partition_pack: p must be in [1, {PACK_MAX_P}]")
    n = keys.numel()
    dev = keys.device
    keys = keys.contiguous()
    row_bytes = 0
    fused_rows = False
    if vals is not None:
        if vals.shape[0] != n:
            raise ValueError("partition_pack: vals rows != keys")
        vals = vals.contiguous()
        row_bytes = (vals[0].numel() if n else 0) * vals.element_size()
        fused_rows = row_bytes % 16 == 0 and row_bytes > 0
    need_perm = want_perm or (vals is not None and not fused_rows)
    out_keys = torch.empty(n, dtype=torch.int64, device=dev)
    out_vals = torch.empty_like(vals) if vals is not None else None
    perm = torch.empty(n, dtype=torch.int64, device=dev) if need_perm else None
    counts = torch.empty(p + (2 if want_range else 0), dtype=torch.int64, device=dev)
    lib = native.hip()
    sb = lib.mp4x_partition_pack_scratch_bytes(n, p)
    scratch = torch.empty(max(sb, 1), dtype=torch.uint8, device=dev)
    check(lib.mp4x_partition_pack(keys.data_ptr(), vals.data_ptr() if fused_rows else None, n, row_bytes, p,
                                  out_keys.data_ptr(), out_vals.data_ptr() if fused_rows else None,
                                  perm.data_ptr() if perm is not None else None, counts.data_ptr(),
                                  counts.data_ptr() + 8 * p if want_range else None,
                                  scratch.data_ptr(), sb, stream_ptr(stream)), "mp4x_partition_pack")
    if vals is not None and not fused_rows and n:
        gather_rows(vals.view(n, -1), perm, out=out_vals.view(n, -1), stream=stream)
    return out_keys, out_vals, counts, perm


class PackCount(NamedTuple):
    """The first half of K4b (:func:`partition_count`): ``info`` = counts[p] + [min key, max
    key]; ``scratch`` holds the scan the second half (:func:`partition_scatter`) reads."""
    keys: torch.Tensor
    p: int
    info: torch.Tensor
    scratch: torch.Tensor


def partition_count(keys: torch.Tensor, p: int, stream=None) -> PackCount:
    """K4b's histogram + scan: rows per owner ``(uint64)key % p`` and the key range, with no rows
    moved yet (the caller can exchange the counts first)."""
    _dev_check(keys)
    if keys.dtype != torch.int64:
        raise ValueError("partition_count: keys must be int64")
    if not 1 <= p <= PACK_MAX_P:
        raise ValueError(f"partition_count: p must be in [1, {PACK_MAX_P}]")
    n = keys.numel()
    lib = native.hip()
    sb = lib.mp4x_partition_pack_scratch_bytes(n, p)
    scratch = torch.empty(max(sb, 1), dtype=torch.uint8, device=keys.device)
    info = torch.empty(p + 2, dtype=torch.int64, device=keys.device)
    check(lib.mp4x_partition_pack_count(keys.data_ptr(), n, p, info.data_ptr(), info.data_ptr() + 8 * p,
                                        scratch.data_ptr(), sb, stream_ptr(stream)), "mp4x_partition_pack_count")
    return PackCount(keys, p, info, scratch)


def partition_scatter(pc: PackCount, vals: Optional[torch.Tensor], out_vals_ptr: int, out_keys_ptr: int,
                      key_stride: int = 1, stream=None) -> None:
    """K4b's scatter after :func:`partition_count`: rows of ``vals`` (whole 16-byte vectors) to
    device address ``out_vals_ptr`` and keys to ``out_keys_ptr`` (``key_stride`` 2: the key half
    of 16-byte vectors) in stable owner-major order."""
    keys = pc.keys
    n = keys.numel()
    if n == 0:
        return
    _dev_check(keys, vals)
    rb = 0 if vals is None else vals[0].numel() * vals.element_size()
    if rb % 16 or (vals is not None and vals.shape[0] != n):
        raise ValueError("partition_scatter: rows of whole 16-byte vectors, one per key")
    check(native.hip().mp4x_partition_pack_scatter(keys.data_ptr(), vals.data_ptr() if vals is not None else None, n,
                                                   rb, pc.p, out_keys_ptr, int(key_stride),
                                                   out_vals_ptr if vals is not None else None, None,
                                                   pc.scratch.data_ptr(), pc.scratch.numel(), stream_ptr(stream)),
          "mp4x_partition_pack_scatter")


# int64 key sorts: rocPRIM's own dispatch (block sort + merge passes below 1 M items, whatever the
# key width) or forced onesweep (csrc/kernels/sparse.hip OnesweepSort: ~27 us per 8-bit pass at
# 200 k items).  Measured on MI355X (profiles/r6/sparse/sort_ab.jsonl): onesweep wins at <= 16 bits
# from 200 k items and at <= 40 bits from ~1 M items (0.107 vs 0.199 ms at 1 M x 24 bits).
# MP4X_SORT_ALGO=rocprim | onesweep pins one.
SORT_ALGO = os.environ.get("MP4X_SORT_ALGO", "auto").lower()


def sort_algo(n: int, bits: int) -> int:
    """0 = rocPRIM's dispatch, 1 = onesweep, for ``n`` int64 keys over ``bits`` bits."""
    if SORT_ALGO in ("rocprim", "onesweep"):
        return int(SORT_ALGO == "onesweep")
    return 1 if bits <= 16 or (n >= 400_000 and bits <= 40) else 0


def sort_pairs(keys: torch.Tensor, idx: Optional[torch.Tensor] = None, end_bit: Optional[int] = None, stream=None,
               algo: Optional[int] = None):
    """Stable radix sort of int64 (or int32) keys with an int64 payload (default arange).
    ``algo`` (int64 keys): 0 = rocPRIM's choice, 1 = onesweep; None = by key width."""
    _dev_check(keys)
    n = keys.numel()
    if idx is None:
        idx = torch.arange(n, dtype=torch.int64, device=keys.device)
    ko = torch.empty_like(keys)
    io = torch.empty_like(idx)
    lib = native.hip()
    is32 = keys.dtype == torch.int32
    tb = lib.mp4x_sort_pairs_temp_bytes(n, int(is32))
    temp = torch.empty(max(tb, 1), dtype=torch.uint8, device=keys.device)
    eb = end_bit if end_bit is not None else (32 if is32 else 64)
    if is32:
        check(lib.mp4x_sort_pairs_i32key(keys.data_ptr(), ko.data_ptr(), idx.data_ptr(), io.data_ptr(), n, 0, eb,
                                         temp.data_ptr(), tb, stream_ptr(stream)), "mp4x_sort_pairs")
        return ko, io
    if algo is None:
        algo = sort_algo(n, eb)
    check(lib.mp4x_sort_pairs_i64_ex(keys.data_ptr(), ko.data_ptr(), idx.data_ptr(), io.data_ptr(), n, 0, eb, int(algo),
                                     temp.data_ptr(), tb, stream_ptr(stream)), "mp4x_sort_pairs")
    return ko, io


def run_starts(sorted_keys: torch.Tensor, stream=None):
    """Start index of every run of equal keys; returns (starts[n] buffer, nruns device scalar)."""
    _dev_check(sorted_keys)
    n = sorted_keys.numel()
    dev = sorted_keys.device
    starts = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    nruns = torch.zeros(1, dtype=torch.int64, device=dev)
    flags = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    lib = native.hip()
    tb = lib.mp4x_rle_temp_bytes(max(n, 1))
    temp = torch.empty(max(tb, 1), dtype=torch.uint8, device=dev)
    check(lib.mp4x_run_starts(sorted_keys.data_ptr(), n, starts.data_ptr(), nruns.data_ptr(), flags.data_ptr(),
                              temp.data_ptr(), tb, stream_ptr(stream)), "mp4x_run_starts")
    return starts, nruns


def stage_split(keys: torch.Tensor, vals: Optional[torch.Tensor], vals_ptr: int, keys16_ptr: int,
                stream=None) -> None:
    """Sparse exchange staging (see mp4x/parallel/sparse.py): rows of ``vals`` [n, ...] copied to
    device address ``vals_ptr`` and ``keys`` [n] written as 16-byte {key, 0} vectors at
    ``keys16_ptr``, one launch (csrc/kernels/copy.hip k_stage_split)."""
    n = keys.shape[0]
    if n == 0:
        return
    _dev_check(keys, vals)
    rb = 0 if vals is None else vals[0].numel() * vals.element_size()
    if keys.dtype != torch.int64 or not keys.is_contiguous() or rb % 16 or \
            (vals is not None and (vals.shape[0] != n or not vals.is_contiguous())):
        raise ValueError("stage_split: contiguous int64 keys[n], rows of whole 16-byte vectors")
    check(native.hip().mp4x_stage_split(keys.data_ptr(), vals.data_ptr() if vals is not None else None, n, rb,
                                        vals_ptr if rb else None, keys16_ptr, stream_ptr(stream)), "mp4x_stage_split")


def keys_from16(k16: torch.Tensor, stream=None) -> torch.Tensor:
    """int64 keys of a uint8 [m * 16] region of {key, 0} vectors (the inverse of the key half of
    :func:`stage_split`)."""
    _dev_check(k16)
    m = k16.numel() // 16
    keys = torch.empty(m, dtype=torch.int64, device=k16.device)
    if m:
        check(native.hip().mp4x_keys_from16(k16.data_ptr(), m, keys.data_ptr(), stream_ptr(stream)), "mp4x_keys_from16")
    return keys


def hash_rbk_supported(dtype: torch.dtype, op: int) -> bool:
    """Does the hash reduce-by-key (K5h, csrc/kernels/sparse_hash.hip) serve (dtype, op)?"""
    try:
        dt = dtype_of_torch(dtype)
    except Exception:   # noqa: BLE001
        return False
    return bool(native.hip().mp4x_hash_rbk_supported(int(dt), int(op)))


def hash_reduce_by_key(keys: torch.Tensor, vals: torch.Tensor, op: int, stream=None):
    """K5h (csrc/kernels/sparse_hash.hip): (unique_keys, reduced_rows, counts) with the keys in
    hash-table order — one hashing pass finds the runs and links each key's rows (instead of the
    sort path's radix sort of the 64-bit keys), and lane groups combine every key's rows in input
    order (runs up to 64 rows: the same values, bit for bit, as :func:`reduce_by_key`).  Every
    reduction except the FIRST rule (then use :func:`reduce_by_key`)."""
    _dev_check(keys, vals)
    n = keys.numel()
    if keys.dtype != torch.int64 or vals.dim() not in (1, 2) or vals.shape[0] != n:
        raise ValueError("hash_reduce_by_key: int64 keys[n] and vals[n] / vals[n, dim]")
    if not hash_rbk_supported(vals.dtype, op):
        raise ValueError(f"hash_reduce_by_key: {vals.dtype} op {op} not supported")
    dev = keys.device
    dim = 1 if vals.dim() == 1 else int(vals.shape[1])
    lib = native.hip()
    sb = lib.mp4x_hash_rbk_scratch_bytes(n)
    scratch = torch.empty(sb + 256, dtype=torch.uint8, device=dev)
    sp = scratch.data_ptr()
    sp += (-sp) % 256                                       # the native layout is 256-byte aligned
    m_flag = torch.empty(2, dtype=torch.int64, device=dev)
    out_keys = torch.empty(n, dtype=torch.int64, device=dev)
    out_vals = torch.empty_like(vals)
    out_count = torch.empty(n, dtype=torch.int32, device=dev)
    check(lib.mp4x_hash_reduce_by_key(int(dtype_of_torch(vals.dtype)), int(op), keys.data_ptr(), n, vals.data_ptr(),
                                      dim, sp, sb, out_keys.data_ptr(), out_vals.data_ptr(),
                                      out_count.data_ptr(), m_flag.data_ptr(), stream_ptr(stream)),
          "mp4x_hash_reduce_by_key")
    m = int(m_flag[0].item())
    return out_keys[:m], out_vals[:m], out_count[:m]


def dense_reduce_by_key(keys: torch.Tensor, vals: Optional[torch.Tensor], op: int, base: int, stride: int, T: int,
                        stream=None):
    """K5d (csrc/kernels/sparse_hash.hip): reduce-by-key of DENSE keys — ``k // stride - base`` in
    [0, T) — by direct addressing: (unique_keys ascending, reduced_rows, counts), the same as
    :func:`reduce_by_key` bit for bit and in the same order, with no sort.  None when the keys
    were not dense after all (a key outside the table, two keys on one slot): use
    :func:`reduce_by_key`."""
    _dev_check(keys, vals)
    n = keys.numel()
    if keys.dtype != torch.int64 or (vals is not None and (vals.dim() not in (1, 2) or vals.shape[0] != n)):
        raise ValueError("dense_reduce_by_key: int64 keys[n] and vals[n] / vals[n, dim] (or None)")
    if n == 0 or T < 1 or stride < 1 or base < 0 or (vals is not None and not hash_rbk_supported(vals.dtype, op)):
        return None
    dev = keys.device
    dim = 0 if vals is None else (1 if vals.dim() == 1 else int(vals.shape[1]))
    lib = native.hip()
    sb = lib.mp4x_dense_rbk_scratch_bytes(n, T)
    scratch = torch.empty(sb + 256, dtype=torch.uint8, device=dev)
    sp = scratch.data_ptr()
    sp += (-sp) % 256
    m_flag = torch.empty(2, dtype=torch.int64, device=dev)
    out_keys = torch.empty(n, dtype=torch.int64, device=dev)
    out_vals = torch.empty_like(vals) if vals is not None else None
    out_count = torch.empty(n, dtype=torch.int32, device=dev)
    check(lib.mp4x_dense_reduce_by_key(int(dtype_of_torch(vals.dtype)) if vals is not None else 0, int(op),
                                       keys.data_ptr(), n, vals.data_ptr() if vals is not None else None, dim,
                                       int(base), int(stride), int(T), sp, sb, out_keys.data_ptr(),
                                       out_vals.data_ptr() if vals is not None else None, out_count.data_ptr(),
                                       m_flag.data_ptr(), stream_ptr(stream)), "mp4x_dense_reduce_by_key")
    m, bad = m_flag.tolist()                                # one sync for both
    if bad:
        return None
    return out_keys[:m], (out_vals[:m] if out_vals is not None else None), out_count[:m]


def reduce_by_key(keys: torch.Tensor, vals: Optional[torch.Tensor], op: int, key_bits: Optional[int] = None,
                  stream=None):
    """Deterministic reduce-by-key: returns (unique_keys, reduced_vals, counts), keys ascending.

    Rows with equal keys are combined in their input order (stable sort), so inputs laid out
    rank after rank reduce in rank order.  ``key_bits``: the caller guarantees every key is in
    [0, 2**key_bits) (dense dictionary ids), so the radix sort runs over those bits only
    (8 bits per onesweep pass: 3 passes for 2**21 keys instead of 8 for full int64 keys).
    """
    _dev_check(keys, vals)
    n = keys.numel()
    dev = keys.device
    if n == 0:
        d = vals.shape[1] if vals is not None and vals.dim() == 2 else 1
        ev = None if vals is None else torch.empty((0, d) if vals.dim() == 2 else (0,), dtype=vals.dtype, device=dev)
        return keys.new_empty(0), ev, torch.empty(0, dtype=torch.int32, device=dev)
    if key_bits is not None and not 1 <= int(key_bits) <= 63:
        raise ValueError(f"reduce_by_key: key_bits {key_bits} outside [1, 63]")
    sk, perm = sort_pairs(keys, end_bit=key_bits, stream=stream)
    starts, nruns = run_starts(sk, stream=stream)
    dim = 1 if vals is None or vals.dim() == 1 else int(vals[0].numel())
    out_keys = torch.empty(n, dtype=torch.int64, device=dev)
    out_count = torch.empty(n, dtype=torch.int32, device=dev)
    out_vals = None
    if vals is not None:
        if vals.shape[0] != n:
            raise ValueError("reduce_by_key: vals rows != keys")
        out_vals = torch.empty((n,) + tuple(vals.shape[1:]), dtype=vals.dtype, device=dev)
    dt = dtype_of_torch(vals.dtype) if vals is not None else DType.F32
    check(native.hip().mp4x_segment_reduce_rows(int(dt), int(op), sk.data_ptr(), perm.data_ptr(), starts.data_ptr(),
                                                nruns.data_ptr(), n, n,
                                                vals.data_ptr() if vals is not None else None, dim,
                                                out_keys.data_ptr(),
                                                out_vals.data_ptr() if out_vals is not None else None,
                                                out_count.data_ptr(), stream_ptr(stream)), "mp4x_segment_reduce_rows")
    m = int(nruns.item())
    return out_keys[:m], (out_vals[:m] if out_vals is not None else None), out_count[:m]
