#!/usr/bin/env python3
"""K1 scale (csrc/kernels/reduce.hip k_scale): the 16-byte vector form (aligned tensors) vs the
scalar form (a view one element off 16-byte alignment: the only form before round 6), f32 and
bf16, 256 Mi elements, read + write bytes / device time."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from mp4x.ops import device_ops as K  # noqa: E402

n = 1 << 28
for dt in (torch.float32, torch.bfloat16):
    for off in (0, 1):
        x = torch.randn(n + off, device="cuda").to(dt)[off:]
        y = torch.empty(n + off, device="cuda", dtype=dt)[off:]
        for _ in range(3):
            K.scale_(y, x, 0.5)
        torch.cuda.synchronize()
        ts = []
        for _ in range(20):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            K.scale_(y, x, 0.5)
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b))
        ms = sorted(ts)[10]
        print(json.dumps({"dtype": str(dt), "form": "vector" if off == 0 else "scalar (misaligned)", "n": n,
                          "ms": round(ms, 4), "TBps": round(n * x.element_size() * 2 / (ms * 1e-3) / 1e12, 2)}))
