#!/usr/bin/env python3
"""A/B of the K6 codec kernels' launch grid (csrc/kernels/codec.hip codec_grid): the capped
grid-stride form (mp4x_set_codec_grid(0)) vs the whole grid (1, the default), for the quantise of
1 GiB f32, and the dequant-reduce's quant blocks per wave iteration (mp4x_set_dq_unroll: 1 / 2 / 4,
0 = the default by input count) for 1 / 2 / 4 / 8 fp8 inputs.  Interleaved rounds, identical
outputs."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mp4x.ops import device_ops as K  # noqa: E402
from mp4x.ops import native  # noqa: E402

lib = native.hip()
lib.mp4x_set_codec_grid.argtypes = [ctypes.c_int]
lib.mp4x_set_codec_grid.restype = None
lib.mp4x_set_dq_unroll.argtypes = [ctypes.c_int]
lib.mp4x_set_dq_unroll.restype = None
n = 1 << 28
x = torch.randn(n, device="cuda")
q = torch.empty(n, dtype=torch.uint8, device="cuda")
s = torch.empty(n // 256, device="cuda")
K.quant_fp8(x, q, s)
qs = [q.clone() for _ in range(8)]
ss = [s.clone() for _ in range(8)]
out = torch.empty(n, device="cuda")


def t(fn, it=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(it):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts)[len(ts) // 2]


cases = {"quant_f32": (lambda: K.quant_fp8(x, q, s), n * 5),
         "dequant_1": (lambda: K.dequant_reduce_fp8(out, qs[:1], ss[:1], n), n * 5),
         "dequant_reduce_2": (lambda: K.dequant_reduce_fp8(out, qs[:2], ss[:2], n), n * 6),
         "dequant_reduce_4": (lambda: K.dequant_reduce_fp8(out, qs[:4], ss[:4], n), n * 8),
         "dequant_reduce_8": (lambda: K.dequant_reduce_fp8(out, qs, ss, n), n * 12)}
ref = {}
for rnd in range(2):
    for full, du in ((0, 1), (1, 1), (1, 2), (1, 4), (1, 0)):
        lib.mp4x_set_codec_grid(full)
        lib.mp4x_set_dq_unroll(du)
        for name, (fn, nbytes) in cases.items():
            ms = t(fn)
            o = (q.clone(), s.clone()) if name.startswith("quant") else (out.clone(),)
            same = all(torch.equal(a, b) for a, b in zip(o, ref.setdefault(name, o)))
            print(json.dumps({"round": rnd, "full_grid": full, "dq_unroll": du, "kernel": name, "ms": round(ms, 4),
                              "TBps": round(nbytes / (ms * 1e-3) / 1e12, 2), "same": same}), flush=True)
lib.mp4x_set_codec_grid(1)
lib.mp4x_set_dq_unroll(0)
