#!/usr/bin/env python3
"""A/B of the grid cap of the streaming kernels that launch through grid_for (csrc/kernels/
common.hpp; mp4x_set_grid_max): kMaxGrid = 2048 blocks with a grid-stride loop vs larger caps,
on scale / row gather (K3) / segment copy (K3) / zero suppression (K6b) / sparse staging.
Interleaved rounds; one JSON line per (cap, kernel)."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mp4x.ops import device_ops as K  # noqa: E402
from mp4x.ops import native  # noqa: E402

lib = native.hip()
if not hasattr(lib, "mp4x_set_grid_max"):
    sys.exit("tools/exp/grid_ab.py: the A/B knob mp4x_set_grid_max was removed after the measurement "
             "(profiles/r6/codec/grid_cap_streaming_ab.jsonl); re-add it to common.hpp's grid_for to rerun")
lib.mp4x_set_grid_max.argtypes = [ctypes.c_int64]
lib.mp4x_set_grid_max.restype = None
n = 1 << 28
x = torch.randn(n, device="cuda")
y = torch.empty_like(x)
rows = torch.randn(1_600_000, 64, device="cuda")
idx = torch.randperm(1_600_000, device="cuda")
keys = torch.arange(200_000, device="cuda")
vals = torch.randn(200_000, 64, device="cuda")
stage = torch.empty(200_000 * 64 * 4 + 200_000 * 16 + 256, dtype=torch.uint8, device="cuda")
sparse_x = x * (torch.rand(n, device="cuda") < 0.1)


def t(fn, it=20):
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


segs = [(i * (n // 8), i * (n // 8), n // 8) for i in range(8)]
base = stage.data_ptr() + (-stage.data_ptr()) % 256
cases = {
    "scale_1GiB": (lambda: K.scale_(y, x, 0.5), n * 8),
    "gather_rows_1.6Mx256B": (lambda: K.gather_rows(rows, idx), 1_600_000 * 256 * 2),
    "segment_copy_1GiB_8segs": (lambda: K.segment_copy_(y, x, segs), n * 8),
    "stage_split_200kx256B": (lambda: K.stage_split(keys, vals, base, base + 200_000 * 256), 200_000 * 272 * 2),
    "zs_encode_1GiB_10pct": (lambda: K.zs_encode(sparse_x), n * 4),
}
for rnd in range(2):
    for cap in (2048, 16384, 1 << 20):
        lib.mp4x_set_grid_max(cap)
        for name, (fn, nbytes) in cases.items():
            try:
                ms = t(fn)
                print(json.dumps({"round": rnd, "grid_cap": cap, "kernel": name, "ms": round(ms, 4),
                                  "TBps": round(nbytes / (ms * 1e-3) / 1e12, 2)}), flush=True)
            except Exception as e:   # noqa: BLE001
                print(json.dumps({"round": rnd, "grid_cap": cap, "kernel": name, "error": str(e)[:200]}), flush=True)
lib.mp4x_set_grid_max(0)
