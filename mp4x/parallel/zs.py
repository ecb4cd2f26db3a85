"""Lossless zero-suppression wire codec (kernel K6b) and its CPU twin.

Reference: ``compress=true`` wraps every Kryo stream in lossless Deflate
(J/operand/DoubleOperand.java:267-277).  On device tensors the lossless codec is zero
suppression: per 256-element block a 256-bit non-zero mask (4 × int64; bit l of mask word k <-> word
4l + k, the layout of one wave whose lane l loads words 4l..4l+3), a non-zero count and the
compacted non-zero words in element order.  Dense data costs 1/8 bit per element of masks plus the
counts, so ``DeviceEngine`` only sends encoded chunks when they are smaller than raw.

The CPU twin produces the identical format with torch ops so the gloo / loopback tests run
the same schedule without a GPU.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import torch

BLOCK = 256
_INT_OF_WIDTH = {1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}
_LANE_BITS = None


def _lane_weights():
    global _LANE_BITS
    if _LANE_BITS is None:
        w = torch.ones(64, dtype=torch.int64)
        for i in range(64):
            w[i] = (1 << i) if i < 63 else -(1 << 63)
        _LANE_BITS = w
    return _LANE_BITS


def nblocks(n: int) -> int:
    return (n + BLOCK - 1) // BLOCK


def encoded_bytes(n: int, nnz: int, elem: int) -> int:
    """Wire bytes of one chunk: masks + counts + non-zero words."""
    nb = nblocks(n)
    return nb * 32 + nb * 4 + nnz * elem


def encode(x: torch.Tensor, chunks: Sequence[Tuple[int, int]]):
    """-> (masks int64[4*nblk], counts int32[nblk], vals[nnz], nnz per chunk, blk_start)."""
    if x.is_cuda:
        from ..ops.device_ops import zs_encode
        return zs_encode(x, list(chunks))
    x = x.reshape(-1)
    bits = x.view(_INT_OF_WIDTH[x.element_size()])
    ms, cs, vs, nnz, bs = [], [], [], [], [0]
    w = _lane_weights()
    for s, ln in chunks:
        nb = nblocks(ln)
        pad = torch.zeros(nb * BLOCK, dtype=bits.dtype)
        pad[:ln] = bits[s:s + ln]
        nz = (pad != 0).view(nb, 64, 4).transpose(1, 2)      # mask k, bit l <-> word 4l + k
        ms.append((nz.long() * w).sum(-1).reshape(-1))
        cs.append(nz.sum((1, 2)).to(torch.int32))
        v = x[s:s + ln][bits[s:s + ln] != 0]
        vs.append(v)
        nnz.append(int(v.numel()))
        bs.append(bs[-1] + nb)
    cat = lambda xs, dt: torch.cat(xs) if xs else torch.empty(0, dtype=dt)  # noqa: E731
    return cat(ms, torch.int64), cat(cs, torch.int32), cat(vs, x.dtype), nnz, bs


def decode(masks: torch.Tensor, counts: torch.Tensor, vals: torch.Tensor, chunks: Sequence[Tuple[int, int]],
           out: torch.Tensor) -> torch.Tensor:
    """Expand chunk j (concatenated masks / counts / vals, chunk order) into out[s_j : s_j + len_j]."""
    if out.is_cuda:
        from ..ops.device_ops import zs_decode
        return zs_decode(masks, counts, vals.contiguous(), list(chunks), out)
    o = out.reshape(-1)
    lanes = torch.arange(64, dtype=torch.int64)
    mb = 0
    vo = 0
    for s, ln in chunks:
        nb = nblocks(ln)
        m = masks[4 * mb:4 * (mb + nb)]
        nz = ((m[:, None] >> lanes) & 1).bool().view(nb, 4, 64).transpose(1, 2).reshape(-1)[:ln]
        k = int(nz.sum())
        seg = torch.zeros(ln, dtype=o.dtype)
        seg[nz] = vals[vo:vo + k]
        o[s:s + ln] = seg
        vo += k
        mb += nb
    return out


def split_sizes(bs: List[int], nnz: List[int]):
    """Per-chunk element counts of the three wire streams (masks, counts, vals)."""
    nbs = [bs[j + 1] - bs[j] for j in range(len(nnz))]
    return [4 * b for b in nbs], nbs, list(nnz)
