#!/usr/bin/env python3
"""Micro-benchmark of the mp4x CDNA4 kernels vs the HBM roofline and vs PyTorch.

Reports achieved bandwidth (bytes moved / time) per kernel.  Used under rocprofv3 for the
profiles in profiles/.  Interleaves variants in one process (cdna guide §5.4 rule 24).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from mp4x.operators import OpCode  # noqa: E402
from mp4x.ops import device_ops as K  # noqa: E402


def timeit(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(iters):
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=1024, help="per-input size in MiB")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--variants", action="store_true", help="A/B the K1 kernel variants (interleaved rounds)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    n = a.mb * (1 << 20) // 4
    res = {}
    xs = [torch.randn(n, device=dev) for _ in range(8)]
    out = torch.empty_like(xs[0])
    if a.variants:
        from mp4x.ops import native
        lib = native.hip()
        names = {0: "gridstride_u2", 1: "tile", 2: "tile_nt", 3: "tile_nt_u2x"}
        rounds = {}
        for rnd in range(3):
            for v, cap in ((2, 0), (2, 4096), (2, 8192), (2, 16384), (3, 8192)):
                lib.mp4x_set_k1_variant(v)
                lib.mp4x_set_k1_grid(cap)
                for nin in (1, 2, 4, 8):
                    ms = timeit(lambda: K.reduce_(out, xs[:nin], int(OpCode.SUM)), a.iters)
                    rounds.setdefault(f"k1_{names[v]}_grid{cap}_nin{nin}", []).append((nin + 1) * n * 4 / ms / 1e6)
                ms = timeit(lambda: torch.add(xs[0], xs[1], out=out), a.iters)
                rounds.setdefault("torch_add", []).append(3 * n * 4 / ms / 1e6)
        for k, v in rounds.items():
            print(f"{k:28s} GB/s median {sorted(v)[1]:.0f}  all {[round(x) for x in v]}")
        lib.mp4x_set_k1_variant(2)
        lib.mp4x_set_k1_grid(0)
        return
    for nin in ([2, 8] if a.quick else [1, 2, 4, 8]):
        ms = timeit(lambda: K.reduce_(out, xs[:nin], int(OpCode.SUM)), a.iters)
        nbytes = (nin + 1) * n * 4
        res[f"k1_reduce_f32_nin{nin}"] = {"ms": ms, "GBps": nbytes / ms / 1e6}
        if nin == 2:
            ms_t = timeit(lambda: torch.add(xs[0], xs[1], out=out), a.iters)
            res["torch_add_f32"] = {"ms": ms_t, "GBps": nbytes / ms_t / 1e6}
    # bf16
    xb = [x.to(torch.bfloat16) for x in xs[:4]]
    ob = torch.empty_like(xb[0])
    ms = timeit(lambda: K.reduce_(ob, xb, int(OpCode.SUM)), a.iters)
    res["k1_reduce_bf16_nin4"] = {"ms": ms, "GBps": 5 * n * 2 / ms / 1e6}
    # copy (D2D) baseline
    ms = timeit(lambda: out.copy_(xs[0]), a.iters)
    res["torch_copy_f32"] = {"ms": ms, "GBps": 2 * n * 4 / ms / 1e6}
    # fp8 codec
    q = torch.empty(n, dtype=torch.uint8, device=dev)
    s = torch.empty((n + 255) // 256, device=dev)
    ms = timeit(lambda: K.quant_fp8(xs[0], q, s), a.iters)
    res["k6_quant_fp8_f32"] = {"ms": ms, "GBps": (n * 4 + n) / ms / 1e6}
    qs = [q] * 8
    ss = [s] * 8
    ms = timeit(lambda: K.dequant_reduce_fp8(out, qs, ss, n), a.iters)
    res["k6_dequant_reduce_fp8_nin8"] = {"ms": ms, "GBps": (8 * n + n * 4) / ms / 1e6}
    # sparse K4/K5 pipeline: 8 ranks' worth of rows (1.6M x 64 f32) reduced by key
    keys = torch.randint(0, 400_000, (1_600_000,), device=dev, dtype=torch.int64)
    vals = torch.randn(1_600_000, 64, device=dev)
    ms = timeit(lambda: K.reduce_by_key(keys, vals, int(OpCode.SUM)), max(3, a.iters // 4))
    res["k5_reduce_by_key_1.6Mx64"] = {"ms": ms, "GBps": (vals.numel() * 4 * 2 + keys.numel() * 8 * 4) / ms / 1e6}
    # the same keys as dense dictionary ids (< 2**19): the radix sort covers 19 bits (3 passes, not 8)
    ms = timeit(lambda: K.reduce_by_key(keys, vals, int(OpCode.SUM), key_bits=19), max(3, a.iters // 4))
    res["k5_reduce_by_key_1.6Mx64_bits19"] = {"ms": ms,
                                              "GBps": (vals.numel() * 4 * 2 + keys.numel() * 8 * 4) / ms / 1e6}
    idx = torch.randperm(1_600_000, device=dev)
    ms = timeit(lambda: K.gather_rows(vals, idx), a.iters)
    res["k3_gather_rows_1.6Mx64"] = {"ms": ms, "GBps": vals.numel() * 4 * 2 / ms / 1e6}
    # K4 owner partition of one rank's map (200k keys x 64 f32) for p = 8: sort path vs fused K4b
    pk = torch.randint(0, 1 << 62, (200_000,), device=dev, dtype=torch.int64)
    pv = torch.randn(200_000, 64, device=dev)

    def sort_path():
        dest, _ = K.key_owner(pk, 8)
        _, perm = K.sort_pairs(dest, end_bit=3)
        K.gather_rows(pk.view(-1, 1), perm)
        K.gather_rows(pv, perm)

    ms = timeit(sort_path, a.iters)
    res["k4_owner_sort_gather_200kx64_p8"] = {"ms": ms, "GBps": pv.numel() * 4 * 2 / ms / 1e6}
    ms = timeit(lambda: K.partition_pack(pk, pv, 8), a.iters)
    res["k4b_partition_pack_200kx64_p8"] = {"ms": ms, "GBps": pv.numel() * 4 * 2 / ms / 1e6}
    # K6b lossless zero suppression, 256 MiB f32 at 5 % and 100 % density
    zn = 64 << 20
    for dens in (0.05, 1.0):
        zx = torch.randn(zn, device=dev)
        if dens < 1:
            zx *= (torch.rand(zn, device=dev) < dens)
        from mp4x.ops import native
        native.hip().mp4x_zs_set_twopass(0)
        ms = timeit(lambda: K.zs_encode(zx), max(3, a.iters // 4))
        res[f"k6b_zs_encode_1pass_256MiB_d{dens}"] = {"ms": ms, "GBps": zn * 4 / ms / 1e6}
        native.hip().mp4x_zs_set_twopass(1)     # the default three-kernel form
        ms = timeit(lambda: K.zs_encode(zx), max(3, a.iters // 4))
        res[f"k6b_zs_encode_256MiB_d{dens}"] = {"ms": ms, "GBps": zn * 4 / ms / 1e6}
        m_, c_, v_, _, _ = K.zs_encode(zx)
        zo = torch.empty_like(zx)
        ms = timeit(lambda: K.zs_decode(m_, c_, v_, [(0, zn)], zo), max(3, a.iters // 4))
        res[f"k6b_zs_decode_256MiB_d{dens}"] = {"ms": ms, "GBps": zn * 4 / ms / 1e6}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
